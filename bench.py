"""Headline benchmark: ResNet-50 amp O2 training images/sec (BASELINE.json), one rank per GPU.

Configuration (BASELINE.json configs[2]): ResNet-50 (v1.5, 25.6 M params), amp O2 (fp16 model,
fp32 BatchNorm + fp32 master weights, dynamic loss scaling), FusedLAMB, SyncBatchNorm (fused
BN+ReLU / BN+add+ReLU, synchronised across all ranks), beforeholiday_amd DistributedDataParallel
over RCCL. Synthetic 224x224 channels_last images, random-init weights, weak scaling
(--batch images per GPU).

    python bench.py --gpus N --steps K --warmup W          (spawns N rank processes itself)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Without ``WORLD_SIZE`` in the environment and ``--gpus N > 1`` the script starts N children of itself
(one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, 127.0.0.1 rendezvous) BEFORE touching HIP, and
exits with their combined status; under torchrun it is one rank. Either way the job asserts that the
process group really has N ranks.

Rank 0 prints ONE json line; ``value`` is the whole-job images/sec over N GPUs; the timed region is
exactly K full training steps (forward, scaled backward with overlapped all-reduce, unscale,
optimizer step, master->model copy) bracketed by barrier + synchronize, max over ranks.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _launch_module():
    """beforeholiday_amd/parallel/launch.py loaded by path: stdlib only, so the parent of a spawned
    job never imports the package (or its HIP library) before its children start."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "_bh_launch", os.path.join(ROOT, "beforeholiday_amd", "parallel", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod

METRIC = "ResNet-50 amp O2 images/sec"
BASELINE_VALUE = None  # BASELINE.json "published" is empty for this metric


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--opt-level", default="O2", choices=["O1", "O2", "O4", "O5"],
                    help="O2: fp16 model + fp32 master weights (reference headline), O5: its bf16 twin; "
                         "O1 / O4: fp32 model with fp16 / bf16 casts around torch functions")
    ap.add_argument("--optimizer", default="lamb", choices=["lamb", "adam", "sgd"])
    ap.add_argument("--no-syncbn", action="store_true")
    ap.add_argument("--message-size", type=int, default=12_500_000,
                    help="DDP bucket size in elements (reference policy; used when --bucket-cap-mb is 0)")
    ap.add_argument("--bucket-cap-mb", type=float, default=-1,
                    help="DDP bucket size in MB (-1: sized per xGMI peer by xgmi_bucket_mb, 0: use --message-size)")
    ap.add_argument("--syncbn-stats", default="allreduce", choices=["allreduce", "allgather"],
                    help="SyncBN forward statistics: one [2C+1] SUM all-reduce, or the reference all_gather + merge")
    ap.add_argument("--diag-steps", type=int, default=3,
                    help="untimed steps AFTER the timed region with collective timing events (comm_ms_per_step)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--trace-warmup", default="", help="write a cProfile table of warmup step 1 to this file")
    ap.add_argument("--autotune", action="store_true",
                    help="MIOpen find (cudnn.benchmark): minutes of first-step tuning on a fresh box and measured "
                         "slower (35.1 ms/step) than the immediate-mode solvers (33.1 ms/step) at batch 256")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-rank code path, e.g. several ranks sharing one GPU)")
    ap.add_argument("--bn-group", default="auto", choices=["auto", "separate", "world", "ipc"],
                    help="auto (default): ipc when every rank is on this node and the IPC setup + probe exchange "
                         "succeed on all ranks, else separate; ipc: SyncBN stats through HIP-IPC peer memory "
                         "(PeerAllReduce: one push + epoch-flag kernel, no RCCL launch per BN layer); separate: "
                         "SyncBN stats on their own RCCL communicator, so a BN all_reduce never queues behind a DDP "
                         "gradient bucket on the same RCCL stream; world: the default process group")
    ap.add_argument("--stem", default="fused", choices=["fused", "unfused"],
                    help="fused: bn1+ReLU+maxpool in one HIP pass; unfused: SyncBN+ReLU then torch max_pool2d")
    ap.add_argument("--conv1x1", default="auto", choices=["auto", "miopen", "gemm"],
                    help="stride-1 1x1 convolution forward / data gradient: hipBLASLt GEMMs on the channels_last "
                         "view, MIOpen, or the faster per shape (auto, timed in the first warmup step)")
    ap.add_argument("--host-scaler", action="store_true",
                    help="dynamic loss scale read on the host every step (the reference's .item() per step); "
                         "default: device-resident scale, overflow skipped by the fused optimizer's noop flag")
    ap.add_argument("--graph", default="auto", choices=["auto", "off", "on"],
                    help="replay the whole training step as one captured HIP graph (utils/graphs.py capture_checked: "
                         "after capture every rank replays one step and runs one eager step from the same saved "
                         "state, and all ranks keep the graph only if both agree bitwise everywhere, else all run "
                         "eager in this process); auto: on for one rank; on: also for several ranks (the DDP bucket "
                         "all-reduces and the IPC SyncBN exchange, whose epoch lives in device memory, captured); off: "
                         "eager")
    ap.add_argument("--conv3x3", default="auto", choices=["auto", "miopen", "direct"],
                    help="stride-1 3x3 convolution forward / data gradient: the direct MFMA kernel "
                         "(kernels/conv.hip), MIOpen, or the faster per shape (auto)")
    # (same option as utils/gemm_tuning.add_argument, spelled out: the parent of a spawned job must not
    # import the package before its children start)
    ap.add_argument("--gemm-table", default="auto", choices=["auto", "off", "tune"],
                    help="library GEMMs (layer 2-4 1x1 convolutions): auto loads the shipped per-shape hipBLASLt / "
                         "rocBLAS solution table (utils/gemm_tuning.py), tune times every solution of each new "
                         "shape and rewrites the table (offline only), off keeps hipBLASLt's default heuristic")
    return ap.parse_args()


def syncbn_exchange(mode, world):
    """The SyncBN statistics reducer for ``--bn-group`` (see its help) and its name for the JSON line.
    Every rank takes the same branch: the IPC setup and probe agree across ranks before use."""
    if mode in ("auto", "ipc"):
        single_node = int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world
        if single_node or mode == "ipc":
            from beforeholiday_amd.contrib.peer_memory import build_peer_allreduce

            # [2C+1] floats for C <= 2048 channels (ResNet-50's widest BatchNorm)
            red = build_peer_allreduce(capacity=1 << 13)
            if red is not None:
                return red, "ipc"
            if mode == "ipc":
                sys.exit("bench.py: --bn-group ipc, but HIP-IPC peer memory could not be set up on every rank")
        mode = "separate"
    if mode == "separate":
        return dist.new_group(list(range(world))), "rccl-separate"
    return None, "rccl-world"


def main():
    args = parse()
    rc = _launch_module().maybe_spawn(args.gpus)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; run `python bench.py --gpus N` (spawns the "
                 f"ranks) or torchrun with --nproc-per-node N")
    ndev = torch.cuda.device_count()
    if args.backend == "gloo":
        local_rank %= max(1, ndev)  # rehearsal: several ranks may share one GPU
    elif local_rank >= ndev:
        sys.exit(f"bench.py: rank {rank} wants GPU {local_rank} but only {ndev} are visible (RCCL needs one GPU per rank)")
    torch.cuda.set_device(local_rank)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    # Everything from the model on runs on one side stream: DDP registers its gradient hooks there, so the
    # AccumulateGrad nodes of the hooked parameters run on the stream a captured step records (a node made
    # on the default stream stays outside the capture: utils/graphs.py GraphedStep.capture)
    with torch.cuda.stream(torch.cuda.Stream()):
        _train(args, world, rank)


def _train(args, world, rank):
    torch.backends.cudnn.benchmark = args.autotune
    from beforeholiday_amd.utils import gemm_tuning

    gemm_tuned = gemm_tuning.setup(args.gemm_table)

    from beforeholiday_amd import amp, config
    from beforeholiday_amd._native import require_native
    from beforeholiday_amd.models import resnet50, resnet50_fused
    from beforeholiday_amd.optimizers import FusedAdam, FusedLAMB, FusedSGD
    from beforeholiday_amd.parallel import DistributedDataParallel, comm_stats
    from beforeholiday_amd.parallel.distributed import xgmi_bucket_mb
    from beforeholiday_amd.parallel.optimized_sync_batchnorm import set_stats_mode

    require_native("bench")
    if not args.host_scaler:
        config.set(amp_device_scaler=True)  # amp/scaler.py enable_device_mode: no host sync per step
    # the fused mixed-precision LAMB / Adam step (opt-in: amp/_process_optimizer.py): the step reads the scaled
    # fp16 gradients and writes the fp16 model copy itself; the bench never clips through param_groups
    config.set(amp_fused_master_step=True)
    set_stats_mode(args.syncbn_stats)
    config.check_ranks()  # every rank runs the same typed configuration (raises otherwise)
    torch.manual_seed(1234 + rank)
    bn_group, bn_exchange = None, "none"
    if world > 1:
        bn_group, bn_exchange = syncbn_exchange(args.bn_group, world)
    model = (resnet50() if args.no_syncbn else resnet50_fused(process_group=bn_group, channel_last=True,
                                                                   conv1x1_mode=args.conv1x1, conv3x3_mode=args.conv3x3,
                                                                   stem_pool_fused=args.stem == "fused")).cuda()
    model = model.to(memory_format=torch.channels_last)
    global_batch = args.batch * world
    # the whole step as one HIP graph (the loss scale must live on the device: FusedLAMB / FusedSGD with the
    # device scaler, or a static scale -- O4 / O5 -- for FusedAdam, whose lr / step then stay on the device
    # too: capturable=True). Several ranks capture too when every collective inside the step can be captured:
    # the DDP buckets' RCCL all-reduces and the IPC SyncBN exchange (device-resident epoch,
    # tests/test_rccl_world1.py); capture_checked proves the replay against an eager step on every rank first
    # auto captures one rank; several ranks capture with --graph on (the self-check below falls back to eager on a
    # mismatch: with the DDP bucket all-reduces inside the capture the replay measured NOT bitwise equal to the
    # eager step at world 1 with the collectives forced -- tests/test_graph_checked.py -- so auto keeps them eager)
    step_ok = not args.host_scaler and (args.optimizer != "adam" or args.opt_level in ("O4", "O5"))
    use_graph = args.graph == "on" or (args.graph == "auto" and step_ok and world == 1)
    if args.optimizer == "lamb":
        opt = FusedLAMB(model.parameters(), lr=4e-3 * global_batch / 4096, weight_decay=0.01)
    elif args.optimizer == "adam":
        opt = FusedAdam(model.parameters(), lr=1e-3, weight_decay=0.01, capturable=use_graph)
    else:
        opt = FusedSGD(model.parameters(), lr=0.1 * global_batch / 256, momentum=0.9, weight_decay=1e-4)
    model, opt = amp.initialize(model, opt, opt_level=args.opt_level, verbosity=0,
                                keep_batchnorm_fp32=True if args.opt_level in ("O2", "O5") else None)
    grad_bytes = sum(p.numel() * p.element_size() for p in model.parameters())
    if args.bucket_cap_mb < 0:
        cap_mb, first_mb = xgmi_bucket_mb(world, grad_bytes)
    elif args.bucket_cap_mb == 0:
        cap_mb = first_mb = None
    else:
        cap_mb, first_mb = args.bucket_cap_mb, args.bucket_cap_mb / 4
    model = DistributedDataParallel(model, message_size=args.message_size, bucket_cap_mb=cap_mb,
                                    first_bucket_mb=first_mb, gradient_as_bucket_view=True)

    dt = torch.float16 if args.opt_level in ("O1", "O2") else torch.bfloat16
    in_dt = dt if args.opt_level in ("O2", "O5") else torch.float32  # O1/O4 models stay fp32
    x = torch.randn(args.batch, 3, 224, 224, device="cuda", dtype=in_dt).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device="cuda")

    def step():
        out = model(x)
        loss = F.cross_entropy(out, y)
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        opt.step()
        opt.zero_grad()
        return loss

    for i in range(args.warmup):
        tw = time.perf_counter()
        if i == 0 and args.trace_warmup:
            # where the first step's host time goes (MIOpen find / kernel JIT, hipBLASLt heuristics,
            # per-shape A/B timing): cumulative-time table of the slowest calls
            import cProfile
            import pstats

            prof = cProfile.Profile()
            prof.enable()
            step()
            torch.cuda.synchronize()
            prof.disable()
            with open(args.trace_warmup, "w") as f:
                pstats.Stats(prof, stream=f).sort_stats("cumulative").print_stats(60)
        else:
            step()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warmup {i + 1}/{args.warmup}: {(time.perf_counter() - tw) * 1e3:.1f} ms",
                  file=sys.stderr, flush=True)
    run = step
    graph_report = {"graph": "eager"}
    if use_graph:
        from beforeholiday_amd.amp._amp_state import _amp_state
        from beforeholiday_amd.utils import capture_checked, training_state

        state = training_state(*_amp_state.loss_scalers, model=model, optimizer=opt)
        run, graph_report = capture_checked(step, state, watch=list(model.parameters())[:4] + list(model.parameters())[-2:],
                                            model=model)
        if rank == 0:
            print(f"[bench] {graph_report}", file=sys.stderr, flush=True)
        run()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    img_s = global_batch * args.steps / elapsed

    # untimed diagnostics after the timed region: how long the compute stream waited on collectives
    comm = {}
    if world > 1 and args.diag_steps > 0:
        comm_stats.reset()
        with comm_stats.collect():
            for _ in range(args.diag_steps):
                step()
        comm = {k: round(v["ms"] / args.diag_steps, 3) for k, v in comm_stats.summary().items()}
        comm["syncbn_calls_per_step"] = sum(v["calls"] for k, v in comm_stats.summary().items()
                                            if k.startswith("syncbn")) // args.diag_steps
    buckets = [round(n * torch.empty((), dtype=d).element_size() / 2 ** 20, 2) for d, n in model.bucket_sizes()]
    if rank == 0:
        print(json.dumps({
            "metric": METRIC if args.opt_level == "O2" else f"ResNet-50 amp {args.opt_level} images/sec",
            "value": round(img_s, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(img_s / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
            "dtype": "fp16" if dt == torch.float16 else "bf16",
            "data": "synthetic 224x224 channels_last images, random-init weights",
            "config": {
                "model": "ResNet-50 amp O2 + FusedLAMB + SyncBatchNorm, DDP"
                if args.optimizer == "lamb" and not args.no_syncbn and args.opt_level == "O2"
                else f"ResNet-50 amp {args.opt_level} + {args.optimizer}" + ("" if args.no_syncbn else " + SyncBatchNorm"),
                "opt_level": args.opt_level,
                "optimizer": {"lamb": "FusedLAMB", "adam": "FusedAdam", "sgd": "FusedSGD"}[args.optimizer],
                "sync_batchnorm": not args.no_syncbn,
                "global_batch": global_batch,
                "batch_per_gpu": args.batch,
                "image_size": 224,
                "parallelism": f"dp{world}",
                "final_loss": round(float(loss.item()), 4),
            },
            "rccl_world": dist.get_world_size() if world > 1 else 1,
            "backend": (args.backend if world > 1 else "none"),
            "ddp_bucket_mb": buckets,
            "syncbn_stats": args.syncbn_stats,
            "syncbn_exchange": bn_exchange,
            "loss_scaler": "host" if args.host_scaler else "device",
            "hip_graph": run is not step,
            "graph_check": graph_report.get("graph"),
            "gemm_table": dict(gemm_tuning.status(), loaded=bool(gemm_tuned)),
            "comm_ms_per_step": comm,
        }), flush=True)
    gemm_tuning.finish(args.gemm_table, rank)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
