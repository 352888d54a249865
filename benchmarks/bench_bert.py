"""BERT-large pretraining step throughput (BASELINE.json configs[3]: BERT-large amp O2 +
FusedLayerNorm + FusedLAMB, DDP, seq 512), one rank per GPU.

Model: Megatron-style BERT-large (24 layers, hidden 1024, 16 heads, FFN 4096, vocab 30522 padded to a
multiple of 128, seq 512) built from beforeholiday_amd.transformer layers with TP=1: FusedLayerNorm,
fused scale-mask-softmax, fused bias-GELU, fused vocab cross-entropy; masked-LM + NSP loss. amp O2
(fp16 model, fp32 master weights in FusedLAMB, dynamic loss scale), DDP over RCCL for N>1.
Synthetic token ids, random-init weights. Prints one JSON line (sequences/s and tokens/s, whole job).

    python benchmarks/bench_bert.py --batch 16 --steps 10 --warmup 3
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16, help="sequences per GPU")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--opt-level", default="O2", choices=["O2", "O5"])
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the step as one HIP graph (utils/graphs.py capture_checked; dropout seeds from "
                         "the device, utils/graph_rng.py); auto = one rank")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI; gloo only to rehearse several ranks on one GPU")
    from beforeholiday_amd.utils import gemm_tuning

    gemm_tuning.add_argument(ap)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":
        local_rank %= max(1, torch.cuda.device_count())  # rehearsal: several ranks may share one GPU
    torch.cuda.set_device(local_rank)
    gemm_tuning.setup(args.gemm_table)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    if args.backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from beforeholiday_amd import amp
    from beforeholiday_amd._native import require_native
    from beforeholiday_amd.models import BertModel, TransformerConfig
    from beforeholiday_amd.optimizers import FusedLAMB

    if "BH_AMP_DEVICE_SCALER" not in os.environ:  # device-resident loss scale (amp/scaler.py), as bench.py
        from beforeholiday_amd import config

        config.set(amp_device_scaler=True)
    from beforeholiday_amd import config

    config.set(amp_fused_master_step=True)  # opt-in fused mixed-precision step (amp/_process_optimizer.py)
    from beforeholiday_amd.parallel import DistributedDataParallel
    from beforeholiday_amd.transformer import parallel_state, tensor_parallel

    require_native("bench_bert")
    parallel_state.initialize_model_parallel(1, 1, default_backend=args.backend)
    tensor_parallel.model_parallel_cuda_manual_seed(1234)
    fp16 = args.opt_level == "O2"
    cfg = TransformerConfig(hidden_size=1024, num_layers=args.layers, num_attention_heads=16, ffn_hidden_size=4096,
                            vocab_size=30592, max_position_embeddings=args.seq, hidden_dropout=args.dropout,
                            attention_dropout=args.dropout, layernorm_epsilon=1e-12, fp16=fp16, bf16=not fp16,
                            masked_softmax_fusion=True, bias_gelu_fusion=True)
    model = BertModel(cfg, num_tokentypes=2, add_binary_head=True, parallel_output=True).cuda()
    nparams = sum(p.numel() for p in model.parameters())
    opt = FusedLAMB(model.parameters(), lr=1e-4, weight_decay=0.01)
    model, opt = amp.initialize(model, opt, opt_level=args.opt_level, verbosity=0)
    if world > 1:
        model = DistributedDataParallel(model)

    g = torch.Generator(device="cuda").manual_seed(rank)
    B, S = args.batch, args.seq
    tokens = torch.randint(0, 30522, (B, S), device="cuda", generator=g)
    types = torch.randint(0, 2, (B, S), device="cuda", generator=g)
    mask = torch.ones(B, S, device="cuda", dtype=torch.long)
    mask[:, int(S * 0.9):] = 0  # padded tail
    labels = torch.randint(0, 30522, (B, S), device="cuda", generator=g)
    loss_mask = (torch.rand(B, S, device="cuda", generator=g) < 0.15).float()
    nsp = torch.randint(0, 2, (B,), device="cuda", generator=g)

    from beforeholiday_amd.utils import graph_rng

    use_graph = args.graph == "on" or (args.graph == "auto" and world == 1)
    if use_graph:
        graph_rng.enable(seed=rank)  # replayable dropout seeds: a per-call salt + a device step seed

    def step():
        graph_rng.new_step()
        lm_loss, nsp_logits = model(tokens, mask, tokentype_ids=types, lm_labels=labels)
        loss = (lm_loss.float() * loss_mask).sum() / loss_mask.sum() + F.cross_entropy(nsp_logits.float(), nsp)
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        opt.step()
        opt.zero_grad()
        return loss

    for _ in range(args.warmup):
        step()
    run = step
    graph_report = {"graph": "eager"}
    if use_graph:
        from beforeholiday_amd.amp._amp_state import _amp_state
        from beforeholiday_amd.utils import capture_checked, training_state

        state = training_state(*_amp_state.loss_scalers, model=model, optimizer=opt) + graph_rng.state_tensors()
        params = list(model.parameters())
        run, graph_report = capture_checked(step, state, watch=params[:4] + params[-2:], model=model)
        if rank == 0:
            print(f"[bench_bert] {graph_report}", file=sys.stderr, flush=True)
        run()
    if os.environ.get("BH_HOST_PROFILE") == "1":  # CPU-side op profile: a blocking op has a long self time
        from torch.profiler import ProfilerActivity, profile
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            for _ in range(3):
                step()
        if rank == 0:
            print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25), flush=True)
    if os.environ.get("BH_HOST_TIMING") == "1":  # host-side time per phase (a sync shows as a long phase)
        import collections
        acc = collections.defaultdict(float)
        torch.cuda.synchronize()
        for _ in range(5):
            t = [time.perf_counter()]
            lm_loss, nsp_logits = model(tokens, mask, tokentype_ids=types, lm_labels=labels)
            t.append(time.perf_counter())
            loss = (lm_loss.float() * loss_mask).sum() / loss_mask.sum() + F.cross_entropy(nsp_logits.float(), nsp)
            t.append(time.perf_counter())
            with amp.scale_loss(loss, opt) as scaled:
                scaled.backward()
                t.append(time.perf_counter())
            t.append(time.perf_counter())
            opt.step()
            t.append(time.perf_counter())
            opt.zero_grad()
            t.append(time.perf_counter())
            torch.cuda.synchronize()
            t.append(time.perf_counter())
            for k, name in enumerate(["forward", "loss", "backward", "amp_exit", "opt_step", "zero_grad", "gpu_drain"]):
                acc[name] += (t[k + 1] - t[k]) * 1e3 / 5
        if rank == 0:
            print(json.dumps({"host_ms": {k: round(v, 3) for k, v in acc.items()}}), flush=True)
    if os.environ.get("BH_SYNC_DEBUG") == "1":  # report every host-synchronising op of the timed steps
        import traceback
        import warnings

        def _show(msg, *a, **k):
            print("SYNC:", msg, "".join(traceback.format_stack(limit=10)[:-2]), flush=True)
        warnings.showwarning = _show
        if os.environ.get("BH_SYNC_DEBUG_ERROR") == "1":  # raise at the first one, with the forward stack
            torch.autograd.set_detect_anomaly(True, check_nan=False)
            torch.cuda.set_sync_debug_mode("error")
            step()
        torch.cuda.set_sync_debug_mode("warn")
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], device="cuda", dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el)
    seqs = B * world * args.steps / el
    if rank == 0:
        print(json.dumps({
            "metric": "BERT-large amp O2 pretraining sequences/sec", "value": round(seqs, 2), "unit": "sequences/sec",
            "tokens_per_sec": round(seqs * S, 1), "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
            "dtype": "fp16" if fp16 else "bf16", "data": "synthetic token ids, random-init weights",
            "config": {"model": f"BERT-large ({args.layers} layers, {nparams / 1e6:.0f}M params) + FusedLayerNorm + "
                       "FusedLAMB", "global_batch": B * world, "seq_len": S, "parallelism": f"dp{world}",
                       "final_loss": round(float(loss), 4)},
            "gemm_table": gemm_tuning.status(), "hip_graph": run is not step,
            "graph_check": graph_report.get("graph")}), flush=True)
    gemm_tuning.finish(args.gemm_table, rank)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
