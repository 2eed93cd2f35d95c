#!/usr/bin/env python3
"""Benchmark: MPHF build (BBHash, gamma 2.0) keys/s, device-resident, on N MI355X.

A "step" is one complete MPHF build over the synthetic prefix set already resident
in HBM: FNV-1a key hashes + FNV-1 fingerprints, every BBHash level, level ranks, and
the mph_fp / mph_pos placement — the work of StreamingMPHFBuilder.Build minus file
I/O (/root/reference/pkg/format/mphf_streaming.go:122-213).

  python bench.py [--gpus N --steps K --warmup W --config c3]
  N > 1: torchrun --nproc-per-node N bench.py --gpus N ...  (one process per GPU;
         RCCL communicator owned by libs3imph; torch.distributed/gloo only for the
         rendezvous, barriers and the max-over-ranks time).  `python bench.py --gpus N`
         without torchrun starts that same torchrun itself (before anything touches a
         GPU) and exits with its status; rank 0's JSON line is the output.

Workload: BASELINE.json configs[2] (C3), the largest single-GPU configuration:
100M synthetic prefixes per GPU, avg key 64 B (weak scaling: N GPUs build one MPHF over
N x 100M keys).  At N = 1 lines ride beside it (never `value`): C2 (configs[1], 10M keys,
avg 32 B) as `secondary.c2`, the C5 share of one GPU (25M keys, 1-1024 B) as
`secondary.c5`, and C3 through the north_star's per-level collision-bitmap decomposition
at one rank as `bitmap_n1`.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "s3-inv-db_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# FNV-1a + FNV-1 byte steps per second (x1e12): tools/ubench_fnv.hip mode 3 (the product's
# byte step, s3imph_device.h) from registers at 4 waves/SIMD — the level-0 hash kernel's
# occupancy — on MI355X (profiles/r02_b/ubench_fnv.txt: 4.20 at a measured 2.37 GHz shader
# clock; the hash kernel itself runs at ~2.0 GHz under HBM load).
FNV_STEP_PEAK_T = 4.20

CONFIGS = {
    "c2": dict(kind=0, avg=32, keys_per_gpu=10_000_000,
               workload="C2: 10M synthetic S3 prefixes per GPU, key length uniform 16-48 B (avg 32 B)"),
    "c3": dict(kind=0, avg=64, keys_per_gpu=100_000_000,
               workload="C3: 100M synthetic S3 prefixes per GPU, key length uniform 32-96 B (avg 64 B)"),
    "c4": dict(kind=0, avg=32, keys_per_gpu=125_000_000,
               workload="C4: 125M synthetic prefixes per GPU (1B on 8 GPUs), avg key 32 B"),
    "c5": dict(kind=1, avg=0, keys_per_gpu=25_000_000,
               workload="C5: 25M prefixes per GPU (200M on 8 GPUs), key length log-uniform 1-1024 B"),
}


def stage_alg_bytes(stage: str, n: int, key_bytes: int, info: dict) -> int | None:
    """Algorithmic (minimum) HBM bytes of one launch of a stage, per SURVEY.md §8(d) units.
    Level 0 settles a fraction e^{-1/2} of the keys (gamma = 2); the rest move on."""
    settled = math.exp(-0.5)
    if stage == "hash_count0":  # key bytes + offsets read once; kh + fp written once
        return key_bytes + 8 * (n + 1) + 16 * n
    if stage == "hash_part0":   # P0: key bytes + offsets read once; R20 record (k, f, index) to its super-tile
        return key_bytes + 8 * (n + 1) + 20 * n
    if stage == "scatter0_p0":  # P0: R20 record read from its super-tile slot, written to its 2^14 tile's slot
        return 20 * n + 20 * n
    if stage == "tile0_p0":     # P0: R20 read once; fp_out/pos_out or the next-level record; bits
        return int(20 * n + 16 * settled * n + 24 * (1 - settled) * n + n // 4)
    if stage == "hash_route0":  # sharded build: key bytes + offsets read; (kh, fp, pos) records written once
        return key_bytes + 8 * (n + 1) + 24 * n
    if stage == "scatter0":     # kh + fp read, (kh, fp, pos) record written to its tile bucket
        return 16 * n + 24 * n
    if stage == "tile0":        # bucket records read once; fp_out/pos_out or the next-level
        return int(24 * n + 16 * settled * n + 24 * (1 - settled) * n + n // 4)  # record; bits
    return None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist", action="store_true", help="use the multi-GPU build path even at N=1")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "host"],
                    help="N>1 collectives: RCCL over xGMI (default), or host copies over gloo — a rehearsal "
                         "mode that lets several ranks share one GPU (not a measurement)")
    ap.add_argument("--decomp", default="bitmap", choices=["route", "bitmap"],
                    help="sharded levels (N > 1 or --dist): the north_star's per-level collision bitmap, "
                         "(A, C) planes exchanged over RCCL (bitmap, default; timed with no fallback), or "
                         "records routed to position owners (route)")
    ap.add_argument("--alt", action="store_true",
                    help="N > 1: also time the other decomposition on the same shards (alt_decomposition); "
                         "off by default, so the scaling line depends on the timed decomposition alone")
    ap.add_argument("--no-secondary", action="store_true", help="skip the C2 line beside the C3 headline")
    ap.add_argument("--headline-only", action="store_true",
                    help="skip the lookup / finalize / host_e2e lines (profiling runs)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="rocprofv3 PMC summary (HBM bytes per launch) to attach as roofline.traffic")
    ap.add_argument("--probe-launch", action="store_true",
                    help="(tests) each rank prints its rank / world as JSON and exits before any GPU call")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # One command for N GPUs: start one process per GPU through torchrun and relay its
        # status.  Nothing above this line has touched a GPU (torch is not even imported),
        # and the ranks are child processes, not an exec of this one.
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.probe_launch:
        print(json.dumps({"rank": rank, "world": world, "local_rank": local_rank, "gpus": args.gpus}), flush=True)
        return
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: launch one process per GPU")

    import numpy as np
    import torch

    # Ranks past the device count (a one-GPU box) must share devices; RCCL refuses two ranks
    # on one device, so such a run takes the host transport and is a rehearsal of the N > 1
    # path, never a measurement (its `value` is null).  torch.cuda.device_count() does not
    # initialise the GPU on this image.
    n_dev = max(torch.cuda.device_count(), 1)
    shared = world > n_dev
    transport_note = None
    if shared:
        local_rank = local_rank % n_dev
        if args.transport == "rccl":
            args.transport = "host"
            transport_note = f"host (rehearsal: {world} ranks on {n_dev} GPU(s); RCCL needs a GPU per rank)"
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    torch.cuda.set_device(local_rank)

    import s3imph

    cfg = CONFIGS[args.config]
    plan = s3imph.ShardPlan(rank, world, cfg["keys_per_gpu"] * world)
    blob, offs = s3imph.gen_keys(cfg["kind"], args.seed, cfg["avg"], plan.lo, plan.n_local)
    n = plan.n_local
    key_bytes_local = int(offs[-1])
    dev = f"cuda:{local_rank}"
    d_blob = torch.from_numpy(blob).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    use_dist = world > 1 or args.dist
    fallback = None  # set when the timed build is not the one asked for (reported, never silent)
    if not use_dist:
        ctx = s3imph.DeviceBuilder(local_rank)
        ctx.reserve(n)
        out_cap = n
    else:
        ctx = None
        if args.transport == "rccl":
            ctx, fallback = make_rccl_ctx(s3imph, torch, dist, local_rank, rank, world)
            if ctx is None:
                args.transport = "host"
                transport_note = fallback
        if ctx is None:
            ctx = s3imph.DistBuilder(local_rank, None, rank, world, host_comm=True)
        ctx.set_mode(dist_mode(s3imph, args.decomp))
        ctx.reserve(n, plan.n_global)
        out_cap = ctx.out_cap(plan.n_global)
    d_fp = torch.empty(max(out_cap, 1), dtype=torch.int64, device=dev)
    d_po = torch.empty(max(out_cap, 1), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    if not use_dist:
        def step():
            return ctx.build(d_blob, d_offs, n, d_fp, d_po)
    else:
        def step():
            return ctx.build_shard(d_blob, d_offs, n, plan.lo, d_fp, d_po, out_cap)[2]

    bitmap_error = None
    if use_dist and args.decomp == "bitmap":
        # A strict bitmap build fails (on every rank: dist_agree) when a level misses its
        # size bounds.  Then the routed decomposition — same bytes out — is timed instead,
        # and the line says so (config.decomposition, bitmap_error).
        try:
            step()
        except s3imph.MPHFError as e:
            bitmap_error = str(e)
        fl = torch.tensor([0 if bitmap_error is None else 1], dtype=torch.int64)
        if dist is not None:
            dist.all_reduce(fl)
        if int(fl.item()):
            print(f"[bench] rank {rank}: bitmap decomposition failed ({bitmap_error or 'on another rank'}); "
                  f"timing the routed decomposition", file=sys.stderr)
            args.decomp = "route"
            bitmap_error = bitmap_error or "failed on another rank"
            ctx.set_mode(dist_mode(s3imph, "route"))
    for _ in range(args.warmup):
        step()
    # Timed region: two HIP events per build, around the level-0 hash (the dominant kernel),
    # on the build stream.  Every stage's events cost ~35 us per 1 ms C2 step, so the full
    # stage split comes from a profiled pass after the timed loop.
    ctx.set_profiling(2)
    stage_sum: dict[str, float] = {}

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    info = {}
    for _ in range(args.steps):
        info = step()
        for k, v in ctx.stage_times().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    timed_stages = {k: v / args.steps for k, v in stage_sum.items()}
    ctx.set_profiling(1)
    prof_steps = min(args.steps, 5)
    stage_sum = {}
    for _ in range(prof_steps):
        step()
        for k, v in ctx.stage_times().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    ctx.set_profiling(0)
    dt = (t1 - t0) / args.steps
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        kb = torch.tensor([key_bytes_local], dtype=torch.int64)
        dist.all_reduce(kb)
        key_bytes = int(kb.item())
    else:
        key_bytes = key_bytes_local
    n_global = plan.n_global
    stages = {k: v / prof_steps for k, v in stage_sum.items()}
    # The other decomposition of the sharded levels, timed the same way on the same keys
    # (N > 1 with --alt; beside `value`, never as it).  Off by default: the routed build has
    # never run over RCCL at N > 1, and a line must not depend on it.
    alt = None
    if world > 1 and args.alt and not args.headline_only:
        alt = alt_decomposition(s3imph, ctx, step, args, barrier, dist)

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    mph_len = info.get("mph_bin_len", 0)
    b_alg = key_bytes + 8 * (n_global + 1) + 16 * n_global + mph_len
    result = {
        "metric": "MPHF build keys/s + key-bytes GB/s (device-resident), 1/2/4/8 MI355X",
        # ranks sharing a GPU (host-transport rehearsal) measure nothing: null, and the
        # rehearsal's own rate rides in `rehearsal`
        "value": None if shared else n_global / dt,
        "unit": "keys/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (deterministic splitmix64 prefixes, byte-sorted, distinct)",
        "config": {"workload": cfg["workload"], "config": args.config, "keys": n_global,
                   "transport": (transport_note or args.transport) if world > 1 else None,
                   "decomposition": args.decomp if use_dist else None,
                   "key_bytes": key_bytes, "parallelism": f"shard{world}" if use_dist else "single",
                   "gamma": 2.0, "levels": info.get("num_levels")},
        "key_bytes_GBps": key_bytes / dt / 1e9,
        "stages_ms": {k: round(v, 4) for k, v in stages.items()},  # profiled pass after the timed loop
        "pipeline_roofline": {"bound": "hbm", "alg_bytes": b_alg, "achieved": b_alg / dt / 1e9,
                              "peak": HBM_PEAK_GBPS * world, "unit": "GB/s",
                              "frac": b_alg / dt / 1e9 / (HBM_PEAK_GBPS * world)},
    }
    if shared:
        result["rehearsal"] = {"keys_per_s": n_global / dt, "ranks": world, "gpus": n_dev,
                               "note": "ranks share GPUs through the host transport: checks the N > 1 path end "
                                       "to end, not a measurement"}
    if fallback is not None and not shared:
        # RCCL's communicator could not be made: the GPUs are distinct, so this is a real
        # build on `world` GPUs with collectives staged through host memory (slower than xGMI)
        result["transport_fallback"] = fallback
    if bitmap_error is not None:
        result["bitmap_error"] = bitmap_error
    # Roofline of the dominant kernel (rank 0's stage times, HIP events on the build stream).
    dom = max((k for k in stages if stage_alg_bytes(k, n, key_bytes_local, info) is not None),
              key=lambda k: stages[k], default=None)
    if dom is not None:
        alg = stage_alg_bytes(dom, n, key_bytes_local, info)
        # the dominant kernel's time from the timed region's events when they cover it
        dom_ms = timed_stages.get(dom, stages[dom])
        ach = alg / (dom_ms / 1e3) / 1e9
        traffic = None
        try:
            with open(args.traffic) as f:
                pmc = json.load(f)
            ent = pmc.get(args.config, {}).get(dom)
            if ent and ent.get("n_gpus", 1) == world:
                traffic = ent["hbm_bytes_per_launch"]
        except (OSError, ValueError):
            pass
        try:  # the whole build's counter bytes (tools/gpu.sh pmc), one GPU
            with open(args.traffic) as f:
                pl = json.load(f).get(args.config, {}).get("_pipeline")
            if pl and pl.get("n_gpus", 1) == world and not use_dist:
                result["pipeline_traffic"] = {"hbm_bytes_per_step": pl["hbm_bytes_per_build"],
                                              "read_bytes": pl["read_bytes"], "write_bytes": pl["write_bytes"],
                                              "alg_bytes": b_alg, "ratio": pl["hbm_bytes_per_build"] / b_alg,
                                              "source": os.path.relpath(args.traffic, ROOT)}
        except (OSError, ValueError, KeyError):
            pass
        hbm = {"achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBPS}
        result["roofline"] = {"kernel": dom, "bound": "hbm", **hbm, "traffic": traffic, "alg_bytes": alg,
                              "avg_ms": dom_ms, "timed_region_events": dom in timed_stages}
        if dom in ("hash_count0", "hash_route0", "hash_part0"):
            # The hash is bounded by VALU before HBM: every key byte is one FNV-1a + FNV-1 step
            # (two 64-bit multiplies by the FNV prime); tools/ubench_fnv.hip measured the chip's
            # ceiling for that step from registers.  Its HBM rate rides
            # along in roofline.hbm.
            steps_per_s = key_bytes_local / (dom_ms / 1e3)
            result["roofline"].update({"bound": "valu", "achieved": steps_per_s / 1e12, "peak": FNV_STEP_PEAK_T,
                                       "unit": "T byte-steps/s", "frac": steps_per_s / 1e12 / FNV_STEP_PEAK_T,
                                       "hbm": hbm})
        result["dominant_stage"] = max(stages, key=stages.get)
    if alt is not None:
        result["alt_decomposition"] = {**alt, "keys_per_s": n_global / alt["ms_per_step"] * 1e3
                                       if alt.get("ms_per_step") else None}
    if world == 1 and not use_dist and not args.headline_only:
        result["lookup"] = lookup_rate(ctx, d_blob, d_offs, n, d_fp, d_po)
        result["finalize"] = finalize_rate(ctx, d_blob, d_offs, n)
    if world == 1 and not use_dist and not args.no_secondary:
        # the north_star decomposition on the same keys at one rank (RCCL communicator of one)
        ctx.close()
        del d_fp, d_po
        torch.cuda.empty_cache()
        result["bitmap_n1"] = bitmap_n1_line(s3imph, torch, d_blob, d_offs, n, key_bytes_local, local_rank,
                                             args.steps, args.warmup)
    if world == 1 and not args.headline_only:
        result["host_e2e"] = host_e2e(s3imph, blob, offs, local_rank)
    if world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(s3imph, cfg, args.seed)
    if world == 1 and not use_dist and not args.no_secondary:
        del d_blob, d_offs
        ctx.close()
        torch.cuda.empty_cache()
        sec = {}
        for name in ("c2", "c5"):
            if name != args.config:
                sec[name] = secondary_line(s3imph, local_rank, args.seed, args.steps, args.warmup, name,
                                           extras=name == "c2" and not args.headline_only)
        result["secondary"] = sec
    print(json.dumps(result), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def launch_ranks(n: int, argv: list[str]) -> int:
    """Run this bench as N ranks, one process per GPU, through torchrun on 127.0.0.1 (the
    contract's multi-GPU launch); the ranks inherit stdout, so rank 0's JSON line is this
    command's output.  Returns torchrun's exit status."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
    env.setdefault("OMP_NUM_THREADS", "16")
    print(f"[bench] launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def make_rccl_ctx(s3imph, torch, dist, device: int, rank: int, world: int):
    """This rank's RCCL context, or (None, reason) when the communicator cannot be made on
    some rank — then every rank takes the host transport and the line says so.  A rank whose
    peer failed before joining would wait in ncclCommInitRank forever, so a watchdog ends
    the process if the communicator and the agreement on it take longer than 300 s."""
    import threading
    uid = [s3imph.dist_unique_id() if rank == 0 else None]
    if dist is not None:
        dist.broadcast_object_list(uid, src=0)
    done = threading.Event()

    def watchdog():
        if not done.wait(300):
            print(f"[bench] rank {rank}: RCCL communicator not made within 300 s (a peer failed?)",
                  file=sys.stderr, flush=True)
            os._exit(3)
    threading.Thread(target=watchdog, daemon=True).start()
    ctx, note, ok = None, None, 1
    try:
        ctx = s3imph.DistBuilder(device, uid[0], rank, world)
    except Exception as e:  # noqa: BLE001 - reported, then the fallback
        ok, note = 0, f"host (RCCL communicator failed on rank {rank}: {e})"
        print(f"[bench] rank {rank}: {note}", file=sys.stderr, flush=True)
    if dist is not None:
        t = torch.tensor([ok], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = int(t.item())
    done.set()
    if ok:
        return ctx, None
    if ctx is not None:
        ctx.close()
    return None, note or "host (RCCL communicator failed on another rank)"


def bitmap_n1_line(s3imph, torch, d_blob, d_offs, n: int, key_bytes: int, device: int, steps: int,
                   warmup: int) -> dict:
    """The headline's keys through the north_star decomposition — per-level collision
    bitmap, (A, C) planes, settle — at one rank (an RCCL communicator of one), strict (a
    size-bound miss is an error, not a routed build), timed like the headline: W warm-up
    builds, then K builds between two synchronisations.  Beside `value`, never as it."""
    ctx = s3imph.DistBuilder(device, s3imph.dist_unique_id(), 0, 1)
    try:
        ctx.set_mode(dist_mode(s3imph, "bitmap"))
        ctx.reserve(n, n)
        cap = ctx.out_cap(n)
        d_fp = torch.empty(max(cap, 1), dtype=torch.int64, device=d_blob.device)
        d_po = torch.empty(max(cap, 1), dtype=torch.int64, device=d_blob.device)
        try:
            for _ in range(max(warmup, 1)):
                ctx.build_shard(d_blob, d_offs, n, 0, d_fp, d_po, cap)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                ctx.build_shard(d_blob, d_offs, n, 0, d_fp, d_po, cap)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
        except s3imph.MPHFError as e:
            return {"error": str(e)}
        ctx.set_profiling(1)
        ctx.build_shard(d_blob, d_offs, n, 0, d_fp, d_po, cap)
        st = {k: round(v, 4) for k, v in ctx.stage_times().items()}
        ctx.set_profiling(0)
        return {"decomposition": "bitmap (strict)", "keys": n, "ms_per_step": dt * 1e3, "keys_per_s": n / dt,
                "key_bytes_GBps": key_bytes / dt / 1e9, "steps": steps, "stages_ms": st}
    finally:
        ctx.close()
        torch.cuda.empty_cache()


def dist_mode(s3imph, decomp: str) -> int:
    """The context mode of a timed decomposition: the bitmap one with no fallback to routing
    (a size-bound miss fails the build instead of being timed as the other decomposition)."""
    return s3imph.DIST_BITMAP | s3imph.DIST_STRICT if decomp == "bitmap" else s3imph.DIST_ROUTE


def alt_decomposition(s3imph, ctx, step, args, barrier, dist) -> dict:
    """Time the decomposition bench.py was not asked for (route <-> bitmap) over the same
    shards: min(steps, 5) builds after one warm-up, max over ranks.  The bitmap attempt runs
    with DIST_STRICT so a miss of its size bounds is reported, not timed as routing."""
    import torch
    other = "bitmap" if args.decomp == "route" else "route"
    ctx.set_mode(dist_mode(s3imph, other))
    res = {"decomposition": other}
    dt, err = -1.0, None
    try:
        step()
        k = min(args.steps, 5)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        torch.cuda.synchronize()
        barrier()
        dt = (time.perf_counter() - t0) / k
        res["steps"] = k
    except s3imph.MPHFError as e:  # a bound miss is a global fact: every rank lands here
        err = str(e)
    finally:
        ctx.set_mode(dist_mode(s3imph, args.decomp))
    tt = torch.tensor([dt if err is None else -1.0], dtype=torch.float64)
    fl = torch.tensor([0 if err is None else 1], dtype=torch.int64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dist.all_reduce(fl)
    res["ms_per_step"] = float(tt.item()) * 1e3 if int(fl.item()) == 0 else None
    if err is not None:
        res["error"] = err
    return res


def lookup_rate(ctx, d_blob, d_offs, n: int, d_fp, d_po, reps: int = 5) -> dict:
    """Batched MPHF.Lookup of every member (VerifyMPHF, mphf.go:372-393) against the build
    just timed, device-resident: FNV of each key, level probes, fingerprint check, pos.
    Reported beside `value`; the first call also builds the word-rank table."""
    import torch
    res = torch.empty(n, dtype=torch.int64, device=d_fp.device)
    ctx.lookup(d_blob, d_offs, n, d_fp, d_po, n, res)  # rank table + warm-up
    torch.cuda.synchronize()
    ok = bool(torch.equal(res, torch.arange(n, dtype=torch.int64, device=res.device)))
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.lookup(d_blob, d_offs, n, d_fp, d_po, n, res)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return {"keys_per_s": n / dt, "ms": dt * 1e3, "all_members_found": ok,
            "note": "every member looked up against the last build (device-resident)"}


def finalize_rate(ctx, d_blob, d_offs, n: int, reps: int = 5) -> dict:
    """IndexBuilder.Finalize's other arrays (depth, subtree_end, max_depth_in_subtree, depth
    index; indexbuild.go:393-415,474-503, depthindex.go:32-96) over the same keys in HBM.
    Reported beside `value`, never as it."""
    import torch
    r = ctx.finalize_index(d_blob, d_offs, n)  # scratch + warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = ctx.finalize_index(d_blob, d_offs, n)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return {"keys_per_s": n / dt, "ms": dt * 1e3, "max_depth": r["max_depth"],
            "note": "depth ('/' count), subtree_end, max_depth_in_subtree, depth_offsets/positions; device-resident"}


def host_e2e(s3imph, blob, offs, device: int, reps: int = 3) -> dict:
    """PCIe-inclusive rate of the boundary call a pipeline makes (s3imph_build_host_into):
    pageable host blob/offsets in -> offsets (u16 key lengths) H2D -> blob H2D in pieces, the
    level-0 hash of each piece launched as it lands -> build -> D2H of mph_fp/mph_pos through
    pinned chunk staging + mph.bin marshalled into a caller buffer, all outputs caller-owned
    and reused across calls.  `alloc_api_ms`: s3imph_build_host, which returns mph.bin in a
    fresh malloc'd buffer (Python copies it into bytes).  Reported beside `value`, never as it
    (measurement)."""
    import numpy as np
    n = len(offs) - 1
    out = (np.zeros(n, np.uint64), np.zeros(n, np.uint64))
    mph_buf = np.zeros(s3imph.mph_bin_bound(n), np.uint8)
    s3imph.build_host_into(blob, offs, out, mph_buf, device=device)  # warm (staging buffers, output pages)
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        s3imph.build_host_into(blob, offs, out, mph_buf, device=device)
        best = min(best, time.perf_counter() - t0)
    t0 = time.perf_counter()
    s3imph.build_host(blob, offs, device=device, out=out)
    alloc_ms = (time.perf_counter() - t0) * 1e3
    return {"keys_per_s": n / best, "ms": best * 1e3, "key_bytes_GBps": int(offs[-1]) / best / 1e9,
            "alloc_api_ms": alloc_ms,
            "note": "pageable host memory: offsets as u16 lengths then the blob H2D in 16 pieces with the "
                    "level-0 hash of each piece launched as it lands, build, D2H of fp/pos through pinned "
                    "chunk staging (8 workers), mph.bin into a reused caller buffer; output arrays reused"}


def secondary_line(s3imph, device: int, seed: int, steps: int, warmup: int, name: str = "c2",
                   extras: bool = True) -> dict:
    """C2 (BASELINE configs[1]: 10M keys, avg 32 B) or C5's one-GPU share (configs[4]: 25M
    keys, 1-1024 B log-uniform) on the same GPU: ms/step and keys/s, device-resident, same
    step as the headline; `extras` adds finalize and the host-memory lines.  Reported beside
    `value`, never as it."""
    import numpy as np
    import torch
    cfg = CONFIGS[name]
    n = cfg["keys_per_gpu"]
    blob, offs = s3imph.gen_keys(cfg["kind"], seed, cfg["avg"], 0, n)
    dev = f"cuda:{device}"
    d_blob = torch.from_numpy(blob).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_fp = torch.empty(n, dtype=torch.int64, device=dev)
    d_po = torch.empty(n, dtype=torch.int64, device=dev)
    ctx = s3imph.DeviceBuilder(device)
    ctx.reserve(n)
    for _ in range(warmup):
        ctx.build(d_blob, d_offs, n, d_fp, d_po)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.build(d_blob, d_offs, n, d_fp, d_po)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ctx.set_profiling(1)
    ctx.build(d_blob, d_offs, n, d_fp, d_po)
    stages = {k: round(v, 4) for k, v in ctx.stage_times().items()}
    ctx.set_profiling(0)
    res = {"workload": cfg["workload"], "keys": n, "ms_per_step": dt * 1e3, "keys_per_s": n / dt,
           "key_bytes": int(offs[-1]), "key_bytes_GBps": int(offs[-1]) / dt / 1e9, "steps": steps,
           "stages_ms": stages}
    if extras:
        res["finalize"] = finalize_rate(ctx, d_blob, d_offs, n)
    ctx.close()
    del d_blob, d_offs, d_fp, d_po
    torch.cuda.empty_cache()
    if extras:
        res["host_e2e"] = host_e2e(s3imph, blob, offs, device)
        res["builder_e2e"] = builder_e2e(s3imph, blob, offs, device)
    return res


def builder_e2e(s3imph, blob, offs, device: int, batch: int = 1 << 20, reps: int = 3) -> dict:
    """The builder mirror end to end (StreamingMPHFBuilder: Add x N, then Build(outDir)
    writing the 5 index files): Add feeds the keys to the GPU as they arrive (f3), so
    Build = the last chunk's H2D + the build + fp/pos streamed back and written chunk by
    chunk, beside the prefix files (f2).  `serial_ms` times the same output the serial
    way: build_host (H2D of everything, build, D2H) then s3imph_write_index_files.
    Files go to a temporary directory.  Reported beside `value`, never as it."""
    import shutil
    import tempfile
    import numpy as np
    n = len(offs) - 1
    root = os.environ.get("TMPDIR", "/tmp")
    best = None
    for r in range(reps):
        d = tempfile.mkdtemp(prefix="s3imph_bench_", dir=root)
        try:
            b = s3imph.StreamingMPHFBuilder(d, device)
            if r > 0:  # the first rep runs without the capacity hint (its device arrays grow)
                b.reserve(n, int(offs[-1]))
            t0 = time.perf_counter()
            for lo in range(0, n, batch):
                b.add_batch(blob, offs[lo:min(n, lo + batch) + 1])
            t1 = time.perf_counter()
            b.build(d)
            t2 = time.perf_counter()
            b.close()
            files = sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d))
        finally:
            shutil.rmtree(d, ignore_errors=True)
        if r == 0:
            first = (t1 - t0, t2 - t1)
        elif best is None or t2 - t1 < best[1]:
            best = (t1 - t0, t2 - t1, files)
    serial = float("inf")
    out = (np.zeros(n, np.uint64), np.zeros(n, np.uint64))
    for _ in range(reps):
        d = tempfile.mkdtemp(prefix="s3imph_bench_", dir=root)
        try:
            t0 = time.perf_counter()
            fp, po, mph = s3imph.build_host(blob, offs, device=device, out=out)
            s3imph.write_index_files(d, mph, fp, po, blob, offs)
            serial = min(serial, time.perf_counter() - t0)
        finally:
            shutil.rmtree(d, ignore_errors=True)
    add_s, build_s, files = best
    return {"add_ms": add_s * 1e3, "build_ms": build_s * 1e3, "keys_per_s_build": n / build_s,
            "first_no_hint": {"add_ms": first[0] * 1e3, "build_ms": first[1] * 1e3},
            "files_MB": files / 1e6, "serial_ms": serial * 1e3, "batch_keys": batch,
            "note": "Add in batches (one copy into pooled pinned chunks that DMA to HBM while adding) then "
                    "Build(outDir) incl. the 5 files; best of the capacity-hinted reps; first_no_hint = the "
                    "first builder of the process (no hint: device arrays grow, pinned pool cold); "
                    "serial_ms = build_host + write_index_files on the same set"}


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_cores() -> int:
    """Threads this job may use: the box's CPU share (16 on the GPU pool; os.cpu_count()
    there shows the whole machine) or the affinity mask, whichever is smaller."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def cpu_baseline(s3imph, cfg: dict, seed: int) -> dict:
    """The reference algorithm restated in C (oracle/bbhash_oracle.c), timed on this host.

    - `value`: orc_build_revmap, shaped like StreamingMPHFBuilder.Build (serial FNV Add,
      sequential bbhash.New levels with a reverse map, the Go-map position pass and the
      scatter, mphf_streaming.go:68-261), ONE thread like the reference, on a bounded
      sample of the bench workload: its first 10M keys (~5 s).
    - `all_core`: orc_build_mt on `cores` threads (FNV and placement parallel; the levels
      stay sequential as in bbhash.New without Parallel()), same sample.
    - `sets`: both variants on C1 (wide_single_level 100k -> 100 002 prefixes, the
      reference's benchutil shape) and the reference's 1M bench set
      (generateRealisticPrefixes(1_000_000), mphf_bench_test.go:12-27).
    A reported baseline, not the optimisation target (the GPU kernels' roofline is)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import keysets
    import oracle as O
    lib = O.lib()
    cores = _cpu_cores()

    def timed(blob, offs, reps_min_s: float = 1.0) -> dict:
        n = len(offs) - 1
        out = {}
        for name, fn in (("1_thread", lambda: lib.build_revmap(blob, offs)[0]),
                         ("all_core", lambda: lib.build_mt(blob, offs, threads=cores)[0])):
            reps, t0 = 0, time.perf_counter()
            while True:
                assert fn() == 0
                reps += 1
                el = time.perf_counter() - t0
                if el >= reps_min_s:
                    break
            out[name] = n * reps / el
        return out

    sample_n = min(cfg["keys_per_gpu"], 10_000_000)
    blob, offs = s3imph.gen_keys(cfg["kind"], seed, cfg["avg"], 0, sample_n)
    main = timed(blob[: int(offs[-1])], offs)
    del blob, offs
    sets = {}
    for name, keys in (("c1_wide_single_level_100k", keysets.wide_single_level_prefixes()),
                       ("realistic_1m", keysets.realistic_prefixes(1_000_000))):
        b, o = O.keys_to_blob([k.encode() for k in keys])
        r = timed(b, o, 0.5)
        sets[name] = {"keys": len(o) - 1, "avg_key_B": round(float(o[-1]) / (len(o) - 1), 2),
                      "1_thread_keys_per_s": r["1_thread"], "all_core_keys_per_s": r["all_core"]}
    return {"value": main["1_thread"], "unit": "keys/s", "cores": 1, "kind": "port",
            "sample": f"first {sample_n} keys of the bench workload ({cfg['workload']}), "
                      f"oracle/bbhash_oracle.c orc_build_revmap: serial FNV, sequential levels + reverse map, "
                      f"hash-map positions, scatter (mphf_streaming.go:68-261)",
            "cpu_model": _cpu_model(),
            "all_core": {"value": main["all_core"], "unit": "keys/s", "cores": cores,
                         "note": "orc_build_mt: FNV + placement on all cores, levels sequential"},
            "sets": sets}


if __name__ == "__main__":
    main()
