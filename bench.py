#!/usr/bin/env python3
"""Throughput bench: LiDAR frames/s of the fused ground-removal + cone-detection HIP path.

Workload (BASELINE.json configs[2], and configs[3]'s per-GPU share at 8 GPUs): a batch of
256 synthetic cone-field frames x 65,536 points (64 rings x 1024 columns, xyzi float32,
point_step 16) resident in HBM, simulation params. One step = one cg_run_batch over the
batch. Frames are independent units: each rank processes its own batch (weak scaling, no
data-path collective); the timed region is bracketed by barrier + synchronize and the max
over ranks is reported.

The timed region is one host call: the K steps are enqueued by one cg_run_batches crossing
(step s on engine s mod S and its stream), so the host's per-call latency cannot pace the GPU.

The roofline object prices the dominant kernel by the algorithmic bytes B = 16 N + 20 V + 8 C
+ 64 per frame over its average execution span, which each timed launch stamps
itself (s_memrealtime: first workgroup start to last workgroup end, cg_debug_launch_spans,
armed before the timed region: no host call between the launches). A batch is one launch of
the fused frame kernel, cg_frame_kernel: one workgroup per frame. HIP events on the launch
streams are recorded in a separate, identical pass after it (avg_launch_ms_events).
cpu_baseline times the CPU restatement (oracle/, one core and the job's CPU share, same
frames) on a bounded sample on rank 0.

`--gpus N` without a launcher environment starts N ranks itself (torch.distributed.run on
127.0.0.1, before any GPU call); under a launcher WORLD_SIZE must equal N. At N > 1 the C4
composition (rank 0 scatters the batch over RCCL, gathers per-frame headers) is reported as
`c4_scatter_gather` with its own xGMI roofline; `value` stays the frame-sharded rate.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
HBM_COPY_GBS = 6290.0   # the same guide's measured float4 copy rate (79% of spec), for context only
XGMI_LINK_GBS = 153.0   # one xGMI link, one direction (7 links x ~153 GB/s per GPU)
METRIC = "LiDAR frames/sec @64k pts/frame, 1/2/4/8 MI355X; cluster-set match vs PCL"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--frames", type=int, default=256, help="frames per GPU per step")
    ap.add_argument("--rings", type=int, default=64)
    ap.add_argument("--cols", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the frame-parallel CPU leg (0: the process's CPU share, see cpu_share())")
    ap.add_argument("--single-frame", action="store_true",
                    help="also time C2 single-frame latency at N>1 (always at N=1)")
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 single-frame leg (diagnostic builds)")
    ap.add_argument("--colornet", action="store_true",
                    help="also time the colour classifier service (cg_classify_colors) on re-crops of "
                         "the synthetic frames: one call per frame's cones, and batched calls")
    ap.add_argument("--stamps", action="store_true", help="diagnostic: per-phase in-kernel timing")
    ap.add_argument("--no-c5", action="store_true", help="skip the default C5 single-GPU leg (N=1)")
    ap.add_argument("--c5", action="store_true",
                    help="also time C5's frame shape on this GPU: one 1,048,576-point dense frame "
                         "(128 rings x 8192 columns + clutter) through the large-frame path")
    ap.add_argument("--c5-tiled", action="store_true",
                    help="also time C5 tiled over the ranks: each rank holds a contiguous tile of "
                         "the 1M-point frame; sector keys / counts merged, then (a) survivors gathered to rank 0, "
                         "(b) voxel slabs per rank with a halo exchange (both reported)")
    ap.add_argument("--scatter", action="store_true",
                    help="also time the C4 composition: rank 0 holds the whole batch, RCCL "
                         "scatter to ranks, process, gather per-frame headers (reported separately)")
    ap.add_argument("--no-events", action="store_true", help="skip the HIP-event pass after the timed region")
    ap.add_argument("--sustained-steps", type=int, default=200,
                    help="after the timed region, the same rotation for this many steps in one more "
                         "cg_run_batches call, reported as `sustained` (0: skip)")
    ap.add_argument("--streams", type=int, default=3,
                    help="independent batch engines on their own HIP streams, used round-robin "
                         "by consecutive steps (a step's kernel overlaps the previous step's tail)")
    ap.add_argument("--no-scatter", action="store_true", help="at N>1, skip the C4 scatter/gather leg")
    ap.add_argument("--voxel-order", choices=["pcl", "point"], default="pcl",
                    help="voxel summation order (cg_set_voxel_order): PCL's std::sort permutation (default, "
                         "every voxel bit as the reference) or ascending point order")
    ap.add_argument("--route", type=int, default=0,
                    help="diagnostic: cg_debug_route for the C3 engines")
    ap.add_argument("--dry-run", action="store_true",
                    help="plumbing rehearsal without a GPU: launcher, gloo ranks, barrier + max-over-ranks "
                         "timing and the JSON line (value null); used by the CPU tests")
    args = ap.parse_args()

    # one process per GPU: a plain `bench.py --gpus N` (no launcher environment) starts the N
    # ranks itself, as a child torch.distributed.run, before anything here touches the GPU
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, args.dry_run))
    world = int(world_env or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)

    import numpy as np
    import torch
    import torch.distributed as dist
    # one process per GPU; CG_DIST_BACKEND=gloo only rehearses the N>1 logic with several
    # ranks sharing one GPU (the driver's multi-GPU runs use RCCL)
    backend = os.environ.get("CG_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    # --scatter at one rank: a world-size-1 RCCL group with collectives forced on, so the C4
    # scatter/gather runs under RCCL on a one-GPU box too
    solo_pg = world == 1 and (args.scatter or args.c5_tiled)
    if solo_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or solo_pg:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    import cones_perception_amd as cp
    if solo_pg:
        from cones_perception_amd import dist as cd0
        cd0.force_collectives(True)
    params = cp.load_params("simulation")
    F, N = args.frames, args.rings * args.cols
    # each rank owns frames [rank*F, (rank+1)*F): distinct synthetic scenes per rank
    raw = cp.synth_frames(F, first_frame=rank * F, rings=args.rings, cols=args.cols,
                          threads=min(16, os.cpu_count() or 1))
    # one resident copy of the batch per stream: consecutive in-flight steps read distinct
    # buffers (together larger than the 256 MB Infinity Cache), as a live sensor stream would
    S = max(1, args.streams)
    d_ins = [torch.from_numpy(raw).to(dev) for _ in range(S)]
    # one engine (own output buffers) per stream; dedicated streams: the default stream's
    # handle is 0, which the C-ABI reads as "use the handle's own stream"
    vorder = cp.CG_VOXEL_ORDER_PCL if args.voxel_order == "pcl" else cp.CG_VOXEL_ORDER_POINT
    engines = [cp.BatchEngine(params, device=local).set_voxel_order(vorder) for _ in range(S)]
    if args.route:
        for e_ in engines:
            e_.debug_route(args.route)
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    assert all(st.cuda_stream != 0 for st in streams)
    eng, stream = engines[0], streams[0]
    counter = [0]

    def step(idx=None):
        i = counter[0] if idx is None else idx
        counter[0] += 1
        e, st = engines[i % S], streams[i % S]
        e.run(d_ins[i % S].data_ptr(), F, N, 16, stream=st.cuda_stream)
        return st

    # the K timed steps as one cg_run_batches crossing: step s on engine s % S, its input copy
    # and its stream (the rotation step() follows)
    def queue(k):
        return cp.BatchQueue([engines[i % S] for i in range(k)],
                             [cp.batch_desc(d_ins[i % S].data_ptr(), F, N, 16) for i in range(k)],
                             [streams[i % S].cuda_stream for i in range(k)])

    torch.cuda.synchronize(dev)
    if args.warmup:
        queue(args.warmup).run()
    torch.cuda.synchronize(dev)
    timed = queue(args.steps)
    # each timed launch stamps its own execution span (first workgroup start, last workgroup
    # end: what rocprofv3's kernel trace reports); armed per engine before the region
    spans = torch.zeros((args.steps, SPAN_WORDS), dtype=torch.int64, device=dev)
    spans[:, 0] = 2 ** 63 - 1
    per_eng = [list(range(k, args.steps, S)) for k in range(S)]
    span_bufs = [torch.zeros((max(1, len(ix)), SPAN_WORDS), dtype=torch.int64, device=dev) for ix in per_eng]
    for k in range(S):
        span_bufs[k][:, 0] = 2 ** 63 - 1
    torch.cuda.synchronize(dev)
    for k in range(S):
        engines[k].spans(span_bufs[k].data_ptr(), len(per_eng[k]))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    timed.run()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    counter[0] = args.warmup + args.steps
    for k in range(S):
        if per_eng[k]:
            spans[per_eng[k]] = span_bufs[k][: len(per_eng[k])]
    sp = spans.cpu().numpy()
    spans_ok = bool((sp[:, 0] < 2 ** 63 - 1).all() and (sp[:, 1] > sp[:, 0]).all())
    # HIP events on the launch streams, in an identical untimed pass: with queued launches on
    # three streams a start event fires when its predecessor ends, and the kernel may still
    # wait for CU slots, so this reads above the in-kernel span
    avg_event_ms = None
    if not args.no_events:
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        torch.cuda.synchronize(dev)
        for s_ in range(args.steps):
            st = streams[counter[0] % S]
            evs[s_][0].record(st)
            step()
            evs[s_][1].record(st)
        torch.cuda.synchronize(dev)
        kern_ms = [a.elapsed_time(b) for a, b in evs]
        avg_event_ms = sum(kern_ms) / len(kern_ms)
    step_span_ms = float((sp[:, 1] - sp[:, 0]).mean()) * 1e-5 if spans_ok else avg_event_ms   # 100 MHz ticks
    # the launch's duration as rocprofv3 reports it (dispatch to completion, which includes a
    # queued launch's wait for CU room behind the other streams' launches): each timed launch
    # from the end of the launch before it on its stream (a stream runs its launches in order,
    # so that is when the queue dispatches it; a stream's first launch from the first workgroup
    # start of the region) to its own last workgroup's end, from the timed launches' own in-kernel
    # stamps (no event in the timed region). The in-kernel span (first workgroup start to last
    # end) and the HIP events of the untimed pass are reported beside it. (Round 5 before this:
    # events 120.6 us and rocprofv3 124.9 us over the 20 timed launches, -3.4%.)
    queue_ms = float(queued_durations(sp, S).mean()) * 1e-5 if spans_ok else None
    avg_kernel_ms = queue_ms if queue_ms is not None else (avg_event_ms if avg_event_ms is not None else step_span_ms)
    sustained = None
    if args.sustained_steps > 0:
        sustained = sustained_pass(args, world, dev, engines, queue, S, F, N)

    # algorithmic bytes of one launch, from the frames' own V and C
    res = engines[(counter[0] - 1) % S].results()
    hdr_np = fetch_headers(res, F)
    V = hdr_np[:, 3].astype(np.float64)
    Cn = hdr_np[:, 4].astype(np.float64)
    bytes_per_launch = float((16.0 * N + 20.0 * V + 8.0 * Cn + 64.0).sum())
    achieved_gbs = bytes_per_launch / (avg_kernel_ms * 1e-3) / 1e9

    from cones_perception_amd import dist as cd
    elapsed = cd.max_over_ranks(elapsed, dev)
    census = rank_census(world, local)
    total_frames = F * args.steps * world
    fps = total_frames / elapsed

    if args.stamps and rank == 0:
        torch.cuda.synchronize(dev)
        phase_stamps(engines[0], lambda: step(0), F)
        if S > 1:   # the same batch with the other streams' batches in flight beside it
            phase_stamps(engines[0], lambda: step(0), F,
                         around=lambda: [step(i) for i in range(1, S)], tag="loaded")

    scatter = None
    if args.scatter or (world > 1 and not args.no_scatter):
        scatter = scatter_composition(cp, cd, engines[0], streams[0], raw, F, N, dev, rank, world, args.steps)

    # C5's frame shape on this GPU: by default at N=1 (no collective involved; a failure is
    # reported in the line rather than losing it)
    c5 = None
    if rank == 0 and (args.c5 or (world == 1 and not args.no_c5)):
        try:
            c5 = c5_single_gpu(cp, params, local, order=vorder)
            if vorder != cp.CG_VOXEL_ORDER_POINT:   # the cost of PCL's exact voxel order on C5
                c5["point_order_ms_per_frame"] = c5_single_gpu(cp, params, local, reps=20, batch=1,
                                                               order=cp.CG_VOXEL_ORDER_POINT)["ms_per_frame"]
        except Exception as e:  # noqa: BLE001
            c5 = {"error": repr(e)}

    c5t = None
    if args.c5_tiled:
        c5t = {"gather": c5_tiled(cp, cd, params, local, rank, world)}
        h = c5_tiled(cp, cd, params, local, rank, world, halo=True)
        # the halo form's name only when its code path ran (run_halo_backend); a rank without
        # collectives runs the gather form's backend in point order instead
        ran_halo = str(h.get("halo", {}).get("path", "")).startswith("run_halo_backend")
        c5t["halo" if ran_halo else "gather_backend_point_order"] = h

    single = None
    if rank == 0 and (args.single_frame or world == 1) and not args.no_c2:   # C2: the ROS node's synchronous call
        try:
            single = single_frame_latency(cp, params, raw, local, order=vorder)
        except Exception as e:  # noqa: BLE001
            single = {"error": repr(e)}
    if single is not None and "error" not in single:
        try:
            single["cpp_node"] = single_frame_cpp()
        except Exception as e:  # noqa: BLE001
            single["cpp_node"] = {"error": repr(e)}
    pcie = None
    if rank == 0 and world == 1:   # the same batch from pinned host memory: PCIe-inclusive rate
        try:
            pcie = pcie_inclusive(raw, d_ins, engines, streams, F, N, dev)
        except Exception as e:  # noqa: BLE001
            pcie = {"error": repr(e)}
    elif world > 1 and not args.no_scatter:
        # C4's ingest that scales: every rank copies its own pinned host batch over its own
        # PCIe link (no root), processes it, max over ranks
        pcie = per_rank_ingest(cd, raw, d_ins, engines, streams, F, N, dev, rank, world)
    colornet = None
    if args.colornet and rank == 0:
        colornet = colornet_service(cp, params, raw, local)

    cpu = None
    if rank == 0 and not args.no_cpu:   # rank 0's own batch, timed on this box's host cores
        cpu = cpu_baseline(cp, params, raw, args.cpu_seconds, engines[0], args.cpu_threads, order=vorder)
        if isinstance(c5, dict) and "error" not in c5:
            try:
                c5["cpu_1core"] = c5_cpu(cp, params, c5.pop("_det"), min(args.cpu_seconds, 8.0))
            except Exception as e:  # noqa: BLE001
                c5["cpu_1core"] = {"error": repr(e)}
    if world > 1:   # the other ranks wait for rank 0's CPU leg
        dist.barrier()

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": fps,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"C3/C4: {F} frames x {N} pts per GPU per step (xyzi f32, "
                                   "simulation params), ground_removal + cone_detection fused",
                       "frames_per_gpu": F, "points_per_frame": N, "global_batch": F * world,
                       "parallelism": f"frame-shard x{world}", "streams_per_gpu": S,
                       "launches": "fused frame kernel, one workgroup per frame",
                       "enqueue": "one cg_run_batches call for the timed steps",
                       "voxel_order": args.voxel_order},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic_per_launch(F),
                         "traffic_source": traffic_source(),
                         "kernel": "cg_frame_kernel",
                         "avg_kernel_ms": avg_kernel_ms,
                         "avg_kernel_ms_source": ("timed launches, each from the end of the launch before it on its "
                                                  "stream to its last workgroup's end (s_memrealtime stamps): dispatch "
                                                  "to completion, as rocprofv3" if queue_ms is not None else
                                                  "HIP events on the launch streams, identical untimed pass"
                                                  if avg_event_ms is not None else
                                                  "in-kernel span (s_memrealtime) of the timed launches"),
                         "step_span_ms": step_span_ms,
                         "shader_clock_mhz": shader_clock_mhz(sp) if spans_ok else None,
                         "step_span_ms_max": float((sp[:, 1] - sp[:, 0]).max()) * 1e-5 if spans_ok else None,
                         "step_span_frac": bytes_per_launch / (step_span_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "avg_launch_ms_events": avg_event_ms,
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         # launches on S streams overlap, so per-launch duration counts shared
                         # time S-fold; the aggregate rate is bytes of all launches / wall time
                         "aggregate_achieved": bytes_per_launch * args.steps * world / elapsed / 1e9 / world,
                         "aggregate_frac": bytes_per_launch * args.steps / elapsed / 1e9 / HBM_PEAK_GBS,
                         # the guide's measured streaming rate; frac stays against the spec peak
                         "aggregate_frac_of_measured_copy": bytes_per_launch * args.steps / elapsed / 1e9
                         / HBM_COPY_GBS},
            "cpu_baseline": cpu,
            "host_enqueue_ms_per_step": t_enq / args.steps * 1e3,
            "ranks": census,
        }
        if sustained is not None:
            line["sustained"] = sustained
        if single is not None:
            line["single_frame"] = single
        if colornet is not None:
            line["colornet"] = colornet
        if pcie is not None:
            line["pcie_inclusive" if world == 1 else "c4_per_rank_ingest"] = pcie
        if c5 is not None:
            line["c5_single_gpu"] = {k: v for k, v in c5.items() if not k.startswith("_")}
        if c5t is not None:
            line["c5_tiled"] = c5t
        if scatter is not None:
            line["c4_scatter_gather"] = scatter
        print(json.dumps(line), flush=True)
    if world > 1 or solo_pg:
        dist.destroy_process_group()


def rank_census(world, local):
    """Which devices the ranks run on, as every rank sees it: each rank's device UUID (or PCI
    location), all-gathered over the job's process group. At N > 1 this is the line's proof that
    N ranks ran on N distinct GPUs (two ranks sharing a GPU show distinct_devices 1)."""
    import torch.distributed as dist
    ident = "none (no device)"
    if local is not None:
        import torch
        p = torch.cuda.get_device_properties(local)
        uuid = str(getattr(p, "uuid", "") or "")
        pci = ":".join(str(getattr(p, a)) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id") if hasattr(p, a))
        ident = f"uuid {uuid}" if uuid else (f"pci {pci}" if pci else f"{p.name} #{local}")
    ids = [ident]
    backend = None
    if dist.is_initialized():
        backend = str(dist.get_backend())
        ids = [None] * dist.get_world_size()
        dist.all_gather_object(ids, ident)
    devs = {i for i in ids if not i.startswith("none")}
    return {"ranks_seen": len(ids), "world_size_env": world, "distinct_devices": len(devs),
            "backend": backend, "devices": ids[:16]}


def queued_durations(sp, S):
    """Dispatch-to-completion ticks of launches rotated over S in-order streams, from their
    in-kernel [first workgroup start, last workgroup end] stamps sp (launch i on stream i % S):
    launch i from the end of launch i - S (its stream's previous launch), a stream's first
    launch from the first start of all (every stream's first launch is queued then)."""
    import numpy as np
    sp = np.asarray(sp, np.int64)
    t_first = int(sp[:, 0].min())
    prev = np.array([sp[i - S, 1] if i >= S else t_first for i in range(len(sp))], np.int64)
    return sp[:, 1] - prev


def sustained_pass(args, world, dev, engines, queue, S, F, N):
    """The timed rotation again for --sustained-steps steps in one more cg_run_batches call,
    after the timed region (untimed for `value`). Reports the rate, the aggregate HBM fraction and
    every launch's in-kernel span, split into quarters: per-launch duration drifting upward over
    the run (clock or power) shows as a longer span at equal overlap; queueing shows as more
    launches in flight (overlap depth = sum of spans / wall extent of the quarter)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from cones_perception_amd import dist as cd
    K = args.sustained_steps
    q = queue(K)
    per_eng = [list(range(k, K, S)) for k in range(S)]
    bufs = [torch.zeros((max(1, len(ix)), SPAN_WORDS), dtype=torch.int64, device=dev) for ix in per_eng]
    for b in bufs:
        b[:, 0] = 2 ** 63 - 1
    torch.cuda.synchronize(dev)
    for k in range(S):
        engines[k].spans(bufs[k].data_ptr(), len(per_eng[k]))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    q.run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = cd.max_over_ranks(time.perf_counter() - t0, dev)
    sp = np.zeros((K, SPAN_WORDS), np.int64)
    for k in range(S):
        if per_eng[k]:
            sp[per_eng[k]] = bufs[k][: len(per_eng[k])].cpu().numpy()
    if not ((sp[:, 0] < 2 ** 63 - 1).all() and (sp[:, 1] > sp[:, 0]).all()):
        return {"steps": K, "error": "spans not recorded"}
    res = engines[(K - 1) % S].results()
    hdr = fetch_headers(res, F)
    B = float((16.0 * N + 20.0 * hdr[:, 3].astype(np.float64) + 8.0 * hdr[:, 4].astype(np.float64) + 64.0).sum())
    dur = (sp[:, 1] - sp[:, 0]) * 1e-5          # ms (100 MHz ticks)
    quarters = []
    for a in range(4):
        ix = np.arange(a * K // 4, (a + 1) * K // 4)
        if ix.size < 2:
            continue
        ext = (sp[ix, 1].max() - sp[ix, 0].min()) * 1e-5
        quarters.append({"launches": [int(ix[0]), int(ix[-1])],
                         "span_ms_mean": float(dur[ix].mean()),
                         "shader_clock_mhz": shader_clock_mhz(sp[ix]),
                         "overlap_depth": float(dur[ix].sum() / ext),
                         "ms_per_step": float(ext / ix.size),
                         "aggregate_frac": B * ix.size / (ext * 1e-3) / 1e9 / HBM_PEAK_GBS})
    d0, d3 = quarters[0], quarters[-1]
    drift = d3["span_ms_mean"] / d0["span_ms_mean"] - 1.0
    clk = (d3["shader_clock_mhz"] / d0["shader_clock_mhz"] - 1.0) if d0["shader_clock_mhz"] else None
    deeper = d3["overlap_depth"] / d0["overlap_depth"] - 1.0
    pace = d3["ms_per_step"] / d0["ms_per_step"] - 1.0
    if abs(pace) < 0.03:
        finding = "steady: last quarter's step time within 3% of the first's"
    elif clk is not None and clk < -0.02 and drift > 0.02:
        finding = (f"the shader clock falls {-clk * 100:.1f}% from the first quarter to the last "
                   f"({d0['shader_clock_mhz']:.0f} -> {d3['shader_clock_mhz']:.0f} MHz, s_memtime / s_memrealtime "
                   f"of every workgroup) while per-launch spans grow {drift * 100:.1f}%")
    elif drift > 0.03 and abs(deeper) < 0.03:
        finding = ("per-launch duration drifts upward at equal overlap and the shader clock holds "
                   f"({clk * 100:+.1f}%): not the clock" if clk is not None else
                   "per-launch duration drifts upward at equal overlap")
    elif deeper > 0.03:
        finding = "overlap depth grows (launches queue behind each other)"
    else:
        finding = "step time changes with neither span nor overlap alone"
    return {"steps": K, "value": F * K * world / el, "unit": "frames/s", "ms_per_step": el / K * 1e3,
            "aggregate_frac": B * K / el / 1e9 / HBM_PEAK_GBS,
            "span_ms_mean": float(dur.mean()), "span_ms_p50": float(np.median(dur)),
            "span_ms_max": float(dur.max()),
            "span_frac": B / (float(dur.mean()) * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "quarters": quarters, "span_drift_last_vs_first": drift, "overlap_growth_last_vs_first": deeper,
            "step_time_change_last_vs_first": pace, "shader_clock_change_last_vs_first": clk,
            "shader_clock_mhz": shader_clock_mhz(sp), "finding": finding,
            "includes": f"one more cg_run_batches call of {K} steps after the timed region (same engines, "
                        "inputs and stream rotation), in-kernel spans of every launch"}


SPAN_WORDS = 4   # cg_debug_launch_spans (include/cones_gpu_debug.h CG_SPAN_WORDS)


def shader_clock_mhz(sp):
    """The shader clock of launches from their span records: every workgroup's s_memtime cycles
    over its s_memrealtime ticks (100 MHz), summed over the launches' workgroups."""
    ticks = float(sp[:, 3].sum())
    return float(sp[:, 2].sum()) / ticks * 100.0 if ticks > 0 else None


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, dry_run):
    """Start `n` rank processes of this script under torch.distributed.run on this node
    (rendezvous on 127.0.0.1) and return their exit code. Called before any GPU call."""
    import subprocess
    port = free_port()
    env = dict(os.environ)
    if dry_run:
        env["CG_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd, env=env).returncode


def cpu_share():
    """Threads for the all-core CPU leg and where the number comes from: OMP_NUM_THREADS when the
    environment sets it (the GPU box exports its per-GPU CPU share there, 16, while nproc and the
    affinity mask show every CPU of the machine), else the affinity mask."""
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        return int(omp), "OMP_NUM_THREADS"
    try:
        return len(os.sched_getaffinity(0)), "sched_getaffinity"
    except AttributeError:
        return os.cpu_count() or 1, "os.cpu_count"


def host_info():
    """CPU model, logical CPUs of the machine and of this process's affinity set."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff}


def dry_run(args, world, rank):
    """The launcher and reporting path without device work: gloo ranks, barrier, a timed
    host loop, max over ranks, rank 0's JSON line with value null."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.zeros(1)
    for _ in range(args.warmup):
        t += 1
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t += 1
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        m = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        el = float(m.item())
    census = rank_census(world, None)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "frames/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": el / max(args.steps, 1) * 1e3, "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "none (dry run)",
                          "dry_run": True, "ranks_seen": world, "ranks": census, "host": host_info(),
                          "config": {"workload": "dry run: no device work", "parallelism": f"frame-shard x{world}"}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def _newest_traffic():
    import glob
    got = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*_traffic.json")),
                 key=lambda q: int(os.path.basename(q)[1:].split("_")[0]))
    return got[-1] if got else None


def traffic_per_launch(F):
    """HBM bytes per launch from the newest committed PMC summary (profiles/rNN_traffic.json:
    FETCH_SIZE x2 + WRITE_SIZE per the gfx950 correction), scaled to this launch's frames.
    Not measured in this run: rocprofv3 --pmc passes are separate runs (traffic_source)."""
    p = _newest_traffic()
    if not p:
        return None
    with open(p) as fh:
        t = json.load(fh)
    return t["hbm_bytes_per_frame"] * F


def traffic_source():
    p = _newest_traffic()
    return (f"not measured in this run: {os.path.relpath(p, ROOT)} (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
            "per frame) x frames per launch") if p else None


def fetch_headers(res, F):
    """Copy the per-frame header words of the last batch to host."""
    import ctypes
    import numpy as np
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.zeros((F, 8), np.uint32)
    rc = hip.hipMemcpy(out.ctypes.data, res.d_header, F * 32, 2)   # hipMemcpyDeviceToHost
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed: {rc}")
    return out


STAMP_NAMES = ["start", "pass1 stream", "thresholds", "pass2 codes", "survivor loads + ambiguous",
               "pads + bounds", "voxel minmax", "voxel keys", "voxel sort", "voxel runs",
               "voxel centroids", "cluster adjacency", "cluster forest", "cluster roots", "cluster sizes",
               "cluster keep scan", "cluster order", "csr offsets", "labels", "csr indices",
               "centroids+header"]


def phase_stamps(eng, step, F, around=None, tag="alone"):
    """Diagnostic build of one batch: s_memrealtime stamps at phase boundaries (not timed).
    With `around`, other batches are enqueued on the other streams before and after it."""
    import numpy as np
    from cones_perception_amd import _abi
    lib = _abi.lib()
    _abi.check(lib.cg_debug_stamps(eng.handle, 1))
    if around:
        around()
    step()
    if around:
        around()
    st = np.zeros((F, 32), np.uint64)
    _abi.check(lib.cg_debug_stamps_fetch(eng.handle, st.ctypes.data, F))
    _abi.check(lib.cg_debug_stamps(eng.handle, 0))
    t = st.astype(np.int64)
    # frames whose workgroup left no start stamp (not run by this launch) are left out of every
    # figure: their zero stamps would read as times 0 in the spans and percentiles
    t = t[t[:, 0] > 0]
    if t.shape[0] == 0:
        print("STAMPS " + json.dumps({"tag": tag, "error": "no frame stamped"}), flush=True)
        return
    out = {"tag": tag, "frames_stamped": int(t.shape[0]), "batch_span_us": float((t[:, 20].max() - t[:, 0].min()) / 100.0),
           "wg_end_spread_us": float((t[:, 20].max() - t[:, 20].min()) / 100.0)}
    prev = t[:, 0].copy()
    for i in range(1, 21):
        have = t[:, i] > 0
        if not have.any():
            continue
        d = np.where(have, t[:, i] - prev, 0) / 100.0
        out[STAMP_NAMES[i]] = round(float(np.median(d[have])), 2)
        prev = np.where(have, t[:, i], prev)
    sub = t[:, 21] > 0
    if sub.any():   # wave-0 progress marks inside pass 2 (no barrier): LDS loop, re-reads
        out["pass2a lds loop (wave0)"] = round(float(np.median((t[sub, 21] - t[sub, 2]) / 100.0)), 2)
        out["pass2b re-reads (wave0)"] = round(float(np.median((t[sub, 22] - t[sub, 21]) / 100.0)), 2)
        out["pass2c ballots (wave0)"] = round(float(np.median((t[sub, 3] - t[sub, 22]) / 100.0)), 2)
    sub = (t[:, 23] > 0) & (t[:, 24] > 0)
    if sub.any():   # brute-force clustering: adjacency, parents, flatten, cross-tree unions
        out["clusterA adjacency"] = round(float(np.median((t[sub, 11] - t[sub, 10]) / 100.0)), 2)
        out["clusterB parents"] = round(float(np.median((t[sub, 23] - t[sub, 11]) / 100.0)), 2)
        out["clusterC flatten"] = round(float(np.median((t[sub, 24] - t[sub, 23]) / 100.0)), 2)
        out["clusterD cross unions"] = round(float(np.median((t[sub, 12] - t[sub, 24]) / 100.0)), 2)
    sub = (t[:, 25] > 0) & (t[:, 26] > 0)
    if sub.any():   # survivors (wave 0): its loads and appends, the barrier wait, pads + bounds
        out["gatherA loads (wave0)"] = round(float(np.median((t[sub, 25] - t[sub, 3]) / 100.0)), 2)
        out["gatherB barrier (wave0)"] = round(float(np.median((t[sub, 4] - t[sub, 25]) / 100.0)), 2)
        out["gatherC pads+bounds (wave0)"] = round(float(np.median((t[sub, 26] - t[sub, 4]) / 100.0)), 2)
    life = (t[:, 20] - t[:, 0]) / 100.0
    out["wg_lifetime_us_p10_p50_p90"] = [round(float(np.percentile(life, q)), 1) for q in (10, 50, 90)]
    pct = lambda x: [round(float(np.percentile(x, q)), 1) for q in (0, 10, 50, 90, 100)]
    both = (t[:, 0] > 0) & (t[:, 6] > 0) & (t[:, 5] > 0) & (t[:, 20] > 0)
    if both.sum() > 1:   # split batches: front (0-5) and backend (6-20) workgroups
        t = t[both]
        out["split_frames_stamped"] = int(both.sum())
        base = t[:, 0].min()
        out["front_start_us_pcts"] = pct((t[:, 0] - base) / 100.0)
        out["front_us_pcts"] = pct((t[:, 5] - t[:, 0]) / 100.0)
        out["back_start_us_pcts"] = pct((t[:, 6] - base) / 100.0)
        out["back_us_pcts"] = pct((t[:, 20] - t[:, 6]) / 100.0)
        out["back_end_us_pcts"] = pct((t[:, 20] - base) / 100.0)
    print("STAMPS " + json.dumps(out), flush=True)


def scatter_composition(cp, cd, eng, stream, raw, F, N, dev, rank, world, steps):
    """C4 as composed in SURVEY.md §8e: rank 0 holds all world*F frames in HBM; each step
    scatters F frames to every rank over RCCL, runs the batch, and gathers the per-frame
    result headers back to rank 0. Timed like the main loop (barrier + sync, max over ranks)."""
    import torch
    import torch.distributed as dist
    allf = None
    if rank == 0:
        allf = torch.from_numpy(cp.synth_frames(F * world, first_frame=0, rings=64, cols=N // 64)).to(dev)
    hdr = torch.empty((F, 8), dtype=torch.int32, device=dev)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")   # (once, outside the timed loop)
    hip.hipMemcpyDtoDAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]

    def one():
        mine = cd.scatter_frames(allf, F, raw.shape[1], dev)
        with torch.cuda.stream(stream):
            stream.wait_stream(torch.cuda.current_stream(dev))
            eng.run(mine.data_ptr(), F, N, 16, stream=stream.cuda_stream)
        torch.cuda.current_stream(dev).wait_stream(stream)
        # header words: copy out of the engine's device buffer (int32 view)
        hip.hipMemcpyDtoDAsync(hdr.data_ptr(), eng.results().d_header, F * 32,
                               ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        return cd.gather_headers(hdr)

    one()
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize(dev)
    dist.barrier()
    el = cd.max_over_ranks(time.perf_counter() - t0, dev)
    # the root's egress: every peer's share of the batch leaves over that peer's direct link
    egress = float(F * (world - 1) * raw.shape[1])
    out = {"frames_per_s": F * world * steps / el, "ms_per_step": el / steps * 1e3,
           "backend": dist.get_backend(), "ranks": world,
           "includes": "RCCL scatter of the batch from rank 0, processing, gather of headers"}
    if world > 1:
        ach = egress / (el / steps) / 1e9
        peak = XGMI_LINK_GBS * min(world - 1, 7)
        out["roofline"] = {"bound": "xgmi", "achieved": ach, "peak": peak, "unit": "GB/s", "frac": ach / peak,
                           "bytes_per_step": egress,
                           "peak_basis": f"root egress over {min(world - 1, 7)} direct xGMI links x {XGMI_LINK_GBS} GB/s "
                                         "(assumed: a direct link to every peer, the fully connected 8-GPU "
                                         "xGMI node; the topology is not probed)"}
    else:   # one rank: the scatter is the root's own share, a device-local copy through RCCL
        out["roofline"] = None
        out["note"] = "world size 1 with collectives forced on: RCCL scatter/gather executed, no xGMI traffic"
    return out


def c5_single_gpu(cp, params, device, reps=50, order=None, batch=8, breps=6):
    """C5's frame shape on one GPU, device-resident: one 1M-point dense frame per call of the
    batch engine (large-frame path; the call synchronises once the frame is done)."""
    import numpy as np
    import torch
    raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
    d = torch.from_numpy(raw).to(torch.device("cuda", device))
    eng = cp.BatchEngine(params, device=device)
    if order is not None:
        eng.set_voxel_order(order)
    st = torch.cuda.Stream(torch.device("cuda", device))
    n = raw.shape[1] // 16
    for _ in range(5):
        eng.run(d.data_ptr(), 1, n, 16, stream=st.cuda_stream)
    st.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.run(d.data_ptr(), 1, n, 16, stream=st.cuda_stream)
    st.synchronize()
    dt = (time.perf_counter() - t0) / reps
    r = eng.fetch(0)
    V, C = int(r.voxels.shape[0]), int(r.centroids.shape[0])
    algo = 16.0 * n + 20.0 * V + 8.0 * C + 64.0
    out = {"_det": (raw, r), "ms_per_frame": dt * 1e3, "frames_per_s": 1.0 / dt, "points": n, "K": r.n_kept,
           "M": r.n_filtered, "V": V, "C": C,
           "algorithmic_GBs": algo / dt / 1e9, "hbm_frac": algo / dt / 1e9 / HBM_PEAK_GBS,
           "includes": "device-resident input; one frame per call, replayed from a captured hipGraph: every "
                       "backend launch sized from the frame's N, counts read on the device (no host round "
                       "trip inside the frame); one stream synchronisation per call; backend latency-bound "
                       "(partition levels, leaves, union-find)"}
    if batch > 1:   # a stream of C5 frames: batches of distinct frames, pipelined over two scratch sets
        # the same frame in `batch` distinct buffers: per-frame cost comparable with the leg above
        db = torch.from_numpy(np.repeat(raw, batch, axis=0)).to(torch.device("cuda", device))
        for _ in range(2):
            eng.run(db.data_ptr(), batch, n, 16, stream=st.cuda_stream)
        st.synchronize()
        t0 = time.perf_counter()
        for _ in range(breps):
            eng.run(db.data_ptr(), batch, n, 16, stream=st.cuda_stream)
        st.synchronize()
        bt = (time.perf_counter() - t0) / (breps * batch)
        out["stream_of_frames"] = {"ms_per_frame": bt * 1e3, "frames_per_s": 1.0 / bt, "frames_per_call": batch,
                                   "includes": f"{breps} calls of {batch} 1M-point frames each (copies of the frame above "
                                               "in distinct buffers); frame f+1's front overlaps the host "
                                               "sizing frame f's backend"}
    return out


def c5_cpu(cp, params, det, budget_s):
    """C5's frame through the CPU restatement (oracle/, one core, sequential) for about
    budget_s, and the GPU's result for it (c5_single_gpu) compared bit for bit with the oracle
    in PCL's voxel order."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    from helpers import assert_same_detection
    raw, got = det
    msg = cp.frame_cloud(raw[0])
    n, t0 = 0, time.perf_counter()
    while True:
        ref, _ = O.run(params, msg, O.MODE_PIPELINE)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 50:
            break
    try:
        assert_same_detection(got, ref, "C5")
        exact = True
    except AssertionError:
        exact = False
    fl = O.flann_check(params, msg, O.MODE_PIPELINE)
    return {"ms_per_frame": el / n * 1e3, "frames_per_s": n / el, "cores": 1, "kind": "port",
            "sample": f"{n} C5 frames (1,048,576 points, sequential), {el:.1f} s, oracle/cg_oracle.cpp",
            "gpu_bit_exact_vs_oracle_pcl_order": exact,
            "near_tolerance_pairs": fl["near_tolerance_pairs"],
            "flann_check": {k: fl[k] for k in ("voxels", "queries_differ", "clusters_equal", "near_tolerance_pairs",
                                               "near_tolerance_inside", "closest_inside_ulps")}}


def c5_tiled(cp, cd, params, device, rank, world, reps=20, halo=False):
    """C5 tiled over the ranks (one GPU each): rank r holds points tile_range(r) of the
    1M-point frame in its HBM. Per frame: pass 1 on the tile, one MIN all-reduce of the sector
    keys, the keep decision, one all-gather of count words, one all-gather of survivors to
    rank 0, backend on rank 0. Time = max over ranks; rank 0 checks the tiled result against
    the single-GPU large path on the whole frame."""
    import numpy as np
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", device)
    raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
    n_total = raw.shape[1] // 16
    lo, hi = cd.tile_range(n_total, rank, world)
    tile = torch.from_numpy(np.ascontiguousarray(raw[0, lo * 16: hi * 16])).to(dev)
    eng = cp.BatchEngine(params, device=device)
    run = lambda: cd.run_tiled_frame(eng, tile.data_ptr(), lo, hi - lo, n_total, dev, halo=halo, fetch=False)
    for _ in range(3):
        run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):   # results stay on the device, as in the single-GPU leg
        run()
    torch.cuda.synchronize(dev)
    el = cd.max_over_ranks(time.perf_counter() - t0, dev)
    det = eng.fetch(0) if rank == 0 else None
    out = {"ms_per_frame": el / reps * 1e3, "frames_per_s": reps / el, "ranks": world,
           "points": n_total, "tile_points": hi - lo,
           "includes": ("device-resident tiles; 2 collectives to decide the points, then voxel slabs per rank: "
                        "all-to-all of the survivors, point-to-point halo to the slab below, gather of voxel "
                        "records and component pairs to rank 0, merge there; at one rank one slab: its backend "
                        "(voxel sums in point order) on the survivors where decide left them") if halo else
                       "device-resident tiles; keys and counts merged on the device (cg_tile_*_async), one host read of the gathered counts at N>1; backend on rank 0 (at one rank on its own survivors)"}
    if halo:
        out["halo"] = dict(cd.last_halo_stats)
    if rank == 0:
        full = torch.from_numpy(raw).to(dev)
        ref_eng = cp.BatchEngine(params, device=device)
        if halo:   # each slab sums its voxels in frame-index order
            ref_eng.set_voxel_order(cp.CG_VOXEL_ORDER_POINT)
        ref_eng.run(full.data_ptr(), 1, n_total, 16)
        ref = ref_eng.fetch(0)
        out["identical_to_single_gpu"] = bool(
            det.n_kept == ref.n_kept and det.n_filtered == ref.n_filtered
            and np.array_equal(det.voxels.view(np.uint32), ref.voxels.view(np.uint32))
            and np.array_equal(det.labels, ref.labels)
            and np.array_equal(det.centroids.view(np.uint32), ref.centroids.view(np.uint32)))
        out["C"] = int(det.centroids.shape[0])
    return out


def pcie_inclusive(raw, d_ins, engines, streams, F, N, dev, steps=12):
    """The C3 batch with its input in pinned host memory: every step copies the 256 frames
    over PCIe (on the step's stream) and then processes them; three streams overlap one step's
    copy with another's kernel. Never `value` (the metric is device-resident)."""
    import torch
    host = torch.from_numpy(raw).pin_memory()
    S = len(streams)
    for i in range(2 * S):
        with torch.cuda.stream(streams[i % S]):
            d_ins[i % S].copy_(host, non_blocking=True)
        engines[i % S].run(d_ins[i % S].data_ptr(), F, N, 16, stream=streams[i % S].cuda_stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        with torch.cuda.stream(streams[i % S]):
            d_ins[i % S].copy_(host, non_blocking=True)
        engines[i % S].run(d_ins[i % S].data_ptr(), F, N, 16, stream=streams[i % S].cuda_stream)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    return {"frames_per_s": F / dt, "ms_per_step": dt * 1e3, "h2d_GBs": raw.nbytes / dt / 1e9,
            "includes": "pinned host batch -> device copy (PCIe) + processing per step, 3 streams"}


def per_rank_ingest(cd, raw, d_ins, engines, streams, F, N, dev, rank, world, steps=12):
    """C4 with the frames arriving on every rank's host (each GPU's own sensor feed): each rank
    copies its own pinned batch over its own PCIe link and processes it, pcie_inclusive's loop
    on every rank at once. Timed like the main loop (barrier + sync, max over ranks). The root
    scatter (c4_scatter_gather) sends (N - 1) batches out of one GPU per step; this leg moves no
    frame between GPUs, so it scales with the ranks' PCIe links."""
    import torch
    import torch.distributed as dist
    host = torch.from_numpy(raw).pin_memory()
    S = len(streams)

    def step(i):
        with torch.cuda.stream(streams[i % S]):
            d_ins[i % S].copy_(host, non_blocking=True)
        engines[i % S].run(d_ins[i % S].data_ptr(), F, N, 16, stream=streams[i % S].cuda_stream)

    for i in range(2 * S):
        step(i)
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize(dev)
    dist.barrier()
    el = cd.max_over_ranks(time.perf_counter() - t0, dev)
    dt = el / steps
    return {"frames_per_s": F * world / dt, "ms_per_step": dt * 1e3, "ranks": world,
            "h2d_GBs_per_rank": raw.nbytes / dt / 1e9, "h2d_GBs_total": raw.nbytes * world / dt / 1e9,
            "includes": "every rank: its own pinned host batch -> its device (PCIe) + processing per step, "
                        f"{S} streams; max over ranks; no frame crosses GPUs"}


def colornet_service(cp, params, raw, device, frames=16, reps=50):
    """The colour service (cg_classify_colors, host clouds in, colours out) on the re-crops of
    the first frames' cones: per-frame calls (the node's regime) and one batched call."""
    import numpy as np
    from cones_perception_amd import colornet
    w = np.load(os.path.join(ROOT, "tests", "golden", "dam_net_weights.npy"))
    pipe = cp.ConePipeline(params, device=device)
    per_frame = []
    for f in range(frames):
        det = pipe.cloud_handler(cp.frame_cloud(raw[f]))
        per_frame.append(pipe.recrop(det.centroids))
    clf = colornet.ColorClassifier(w, device=device)
    for crops in per_frame[:2]:
        clf.classify(crops)
    t0 = time.perf_counter()
    for r in range(reps):
        clf.classify(per_frame[r % frames])
    per_call = (time.perf_counter() - t0) / reps
    batch = [c for crops in per_frame for c in crops] * 16
    clf.classify(batch)
    t0 = time.perf_counter()
    for _ in range(10):
        clf.classify(batch)
    bt = (time.perf_counter() - t0) / 10
    n_cones = sum(len(c) for c in per_frame) / frames
    return {"cones_per_frame": n_cones, "points_per_cone": float(np.mean([len(c) for c in batch])),
            "ms_per_frame_call": per_call * 1e3, "batched_cones": len(batch), "batched_ms": bt * 1e3,
            "batched_cones_per_s": len(batch) / bt,
            "includes": "host clouds -> H2D, one workgroup per cone (to_image + dam_net), colours D2H"}


def single_frame_latency(cp, params, raw, device, reps=200, order=None):
    """C2: one 64k frame through the synchronous ROS drop-in call (H2D + kernel + D2H)."""
    pipe = cp.ConePipeline(params, device=device)
    if order is not None:
        pipe.set_voxel_order(order)
    msg = cp.frame_cloud(raw[0])
    for _ in range(10):
        pipe.cloud_handler(msg)
    each = []
    t0 = ti = time.perf_counter()
    for _ in range(reps):
        pipe.cloud_handler(msg)
        tj = time.perf_counter()
        each.append(tj - ti)
        ti = tj
    dt = (ti - t0) / reps
    each.sort()
    return {"latency_ms": dt * 1e3, "latency_p50_ms": each[reps // 2] * 1e3, "latency_p90_ms": each[reps * 9 // 10] * 1e3,
            "frames_per_s": 1.0 / dt,
            "includes": "C2: one 64k-point PointCloud2 in pageable host memory through the synchronous "
                        "ConePipeline.cloud_handler (the split kernel launched first; the host copies the message into "
                        "pinned memory chunk by chunk, publishing each chunk to the workgroup reading "
                        "it over PCIe, its last workgroup writing the packed results into pinned host memory, "
                        "one synchronisation, Python result objects)"}


def single_frame_cpp(reps=500):
    """C2 through the C++ node mirror (cones_perception_amd/host/cones_nodes.hpp, the reference
    nodes' own language): nodes_demo --latency, a child process with its own GPU context."""
    import subprocess
    exe = os.path.join(ROOT, "cones_perception_amd", "lib", "nodes_demo")
    r = subprocess.run([exe, "--latency", str(reps)], capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        return {"error": (r.stderr or r.stdout)[-500:]}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["includes"] = ("C2 in C++: ConePipeline::cloud_handler (cones_nodes.hpp) on one 64k-point PointCloud2 in "
                       "pageable memory: cg_pipeline (split kernel launched, message staged into pinned memory chunk "
                       "by chunk behind it, each chunk workgroup reading its chunk over "
                       "PCIe, results written to pinned host memory, one synchronisation), result vectors")
    return out


def cpu_baseline(cp, params, raw, budget_s, eng, threads, order=None):
    """The CPU restatement (oracle/, -O2) on the first frames of this rank's batch: one core
    sequentially (the reference's regime: one ROS callback at a time), then `threads` cores
    frame-parallel. The same sample's CPU outputs are compared with the GPU's results for
    those frames (the last batch left in `eng`'s device buffers): bit-exact frames,
    identical cluster sets, largest centroid difference."""
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    from helpers import same_bits
    F = raw.shape[0]
    msgs = [cp.frame_cloud(raw[i]) for i in range(F)]
    n = 0
    ref = {}
    t0 = time.perf_counter()
    while True:
        det, _ = O.run(params, msgs[n % F], O.MODE_PIPELINE)
        if n < F:
            ref[n] = det
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s and n >= 20:
            break
    out = {"value": n / el, "unit": "frames/s", "cores": 1, "kind": "port", "host": host_info(),
           "sample": f"{n} frames of this bench's 64k-point synthetic batch (cycling over its "
                     f"first {min(n, F)}), sequential, {el:.1f} s, oracle/cg_oracle.cpp "
                     "(g++ -O2 -ffp-contract=off)"}
    # frame-parallel: ctypes releases the GIL inside the oracle call
    share, share_src = cpu_share()
    if threads <= 0:
        threads = share
    else:
        share_src = "--cpu-threads"
    nt = max(1, threads)
    cnt = [0]
    stop = time.perf_counter() + budget_s / 2

    def worker(k):
        c = 0
        while time.perf_counter() < stop:
            O.run(params, msgs[(k + c * nt) % F], O.MODE_PIPELINE)
            c += 1
        return c

    t1 = time.perf_counter()
    with ThreadPoolExecutor(nt) as ex:
        done = sum(ex.map(worker, range(nt)))
    el2 = time.perf_counter() - t1
    out["all_cores"] = {"value": done / el2, "unit": "frames/s", "cores": nt, "cores_source": share_src,
                        "sample": f"{done} frames, {nt} threads, {el2:.1f} s"}
    # parity of the GPU batch against the same sample: bit for bit against the oracle in the
    # engine's voxel order; cluster index sets and centroids against PCL's order (ORDER_PCL)
    point = order == cp.CG_VOXEL_ORDER_POINT
    exact = sets = order_matters = 0
    maxerr = 0.0
    for i, r in ref.items():
        g = eng.fetch(i)
        st, _ = O.run(params, msgs[i], O.MODE_PIPELINE, O.ORDER_STABLE)
        order_matters += int(not same_bits(st.voxels, r.voxels))
        if point:
            exact += (g.n_kept == st.n_kept and g.n_filtered == st.n_filtered and same_bits(g.voxels, st.voxels)
                      and np.array_equal(g.labels, st.labels) and same_bits(g.centroids, st.centroids)
                      and np.array_equal(g.cluster_indices, st.cluster_indices))
        same_sets = (np.array_equal(g.cluster_offsets, r.cluster_offsets)
                     and np.array_equal(g.cluster_indices, r.cluster_indices))
        sets += same_sets
        if same_sets and g.centroids.size:
            d = np.abs(g.centroids.astype(np.float64) - r.centroids.astype(np.float64))
            maxerr = max(maxerr, float(np.nanmax(d)) if np.isfinite(d).any() else 0.0)
        if not point:
            exact += (same_sets and g.n_kept == r.n_kept and g.n_filtered == r.n_filtered
                      and same_bits(g.voxels, r.voxels) and np.array_equal(g.labels, r.labels)
                      and same_bits(g.centroids, r.centroids))
    # FLANN's own search (restated, oracle SEARCH_FLANN) against the exact radius predicate the
    # device implements, on the same sample (tests/test_flann.py)
    fl = {"frames": 0, "voxels": 0, "queries_differ": 0, "clusters_differ": 0, "near_tolerance_pairs": 0,
          "near_tolerance_inside": 0}
    for i in ref:
        f = O.flann_check(params, msgs[i], O.MODE_PIPELINE)
        fl["frames"] += 1
        fl["clusters_differ"] += int(not f["clusters_equal"])
        for k in ("voxels", "queries_differ", "near_tolerance_pairs", "near_tolerance_inside"):
            fl[k] += f[k]
    out["parity"] = {"frames": len(ref), "reference": "oracle ORDER_PCL (PCL 1.10 VoxelGrid std::sort order)",
                     "near_tolerance_pairs": fl["near_tolerance_pairs"],
                     "near_tolerance_note": "voxel pairs whose float L2_Simple sum lies within 4 ulp of r2 (the "
                                            "only pairs FLANN's float pruning could drop)",
                     "flann_check": fl,
                     "cluster_sets_identical_vs_pcl": int(sets), "max_centroid_abs_err_vs_pcl_m": maxerr,
                     "bit_exact": int(exact),
                     "bit_exact_against": "ORDER_STABLE (point-order mode)" if point else "ORDER_PCL",
                     "voxel_ulp_frames": int(order_matters),
                     "voxel_ulp_frames_note": "frames whose voxel bits differ between PCL's order and point order"}
    return out


if __name__ == "__main__":
    main()
