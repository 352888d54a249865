"""GPT-2-medium tensor-parallel training step throughput (BASELINE.json configs[4]: GPT-2-medium via
beforeholiday_amd.transformer tensor_parallel, fused scaled-masked-softmax + bias-GELU, TP over xGMI).

Model: Megatron-style GPT-2-medium (24 layers, hidden 1024, 16 heads, FFN 4096, vocab 50257 padded to
50304, seq 1024) built from ColumnParallelLinear / RowParallelLinear / VocabParallelEmbedding with
causal flash attention, fused bias-GELU MLP, FusedLayerNorm and vocab-parallel cross-entropy
(reference: apex/transformer/testing/standalone_gpt.py:33-111, tensor_parallel/layers.py:167-780).
amp O5 (bf16 model, fp32 master weights, no loss scale) + FusedAdam: an elementwise optimizer keeps
TP-replicated parameters (LayerNorms, row-parallel biases) bit-identical across TP ranks without a
cross-rank norm. ``--tp`` ranks form one tensor-parallel group; the remaining factor of the world is
data parallel (DDP over the DP group). ``--sp`` turns on Megatron sequence parallelism.
Synthetic token ids, random-init weights. Prints one JSON line (whole-job tokens/s).

    python benchmarks/bench_gpt.py --batch 8 --steps 10 --warmup 3
    python benchmarks/bench_gpt.py --gpus 4 --tp 4 --sp          (spawns the 4 ranks itself)
    python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 benchmarks/bench_gpt.py --gpus 4 --tp 4 --sp
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0,
                    help="ranks; without WORLD_SIZE in the env the script spawns them itself (default: WORLD_SIZE or 1)")
    ap.add_argument("--batch", type=int, default=8, help="sequences per data-parallel rank")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--tp", type=int, default=0, help="tensor-parallel size (default: whole world)")
    ap.add_argument("--sp", action="store_true", help="sequence parallelism inside the TP group")
    ap.add_argument("--opt-level", default="O5", choices=["O2", "O5"])
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the step as one HIP graph (utils/graphs.py capture_checked; dropout seeds from "
                         "the device, utils/graph_rng.py); auto = one rank at O5 (static loss scale: FusedAdam "
                         "keeps lr / step on the device, capturable=True)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI; gloo only to rehearse multi-rank TP/SP on one GPU")
    from beforeholiday_amd.utils import gemm_tuning

    gemm_tuning.add_argument(ap)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import importlib.util

        spec = importlib.util.spec_from_file_location(
            "_bh_launch", os.path.join(ROOT, "beforeholiday_amd", "parallel", "launch.py"))
        launch = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(launch)
        sys.exit(launch.maybe_spawn(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus and args.gpus != world:
        sys.exit(f"bench_gpt.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    if args.backend == "gloo":
        local_rank %= max(1, ndev)  # rehearsal: several ranks may share one GPU
    elif local_rank >= ndev:
        sys.exit(f"bench_gpt.py: rank {rank} wants GPU {local_rank} but only {ndev} are visible")
    torch.cuda.set_device(local_rank)
    gemm_tuning.setup(args.gemm_table)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29534")
    if args.backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = args.tp or world
    assert world % tp == 0, f"world {world} not divisible by tp {tp}"
    assert dist.get_world_size() == world
    dp = world // tp

    from beforeholiday_amd import amp, config

    config.set(amp_fused_master_step=True)  # opt-in fused mixed-precision step (amp/_process_optimizer.py)
    from beforeholiday_amd._native import require_native
    from beforeholiday_amd.models import GPTModel, TransformerConfig, finalize_model_grads
    from beforeholiday_amd.optimizers import FusedAdam
    from beforeholiday_amd.parallel import DistributedDataParallel
    from beforeholiday_amd.transformer import parallel_state, tensor_parallel
    from beforeholiday_amd.transformer.pipeline_parallel.utils import get_ltor_masks_and_position_ids

    require_native("bench_gpt")
    parallel_state.initialize_model_parallel(tp, 1, default_backend=args.backend)
    tensor_parallel.model_parallel_cuda_manual_seed(1234)
    fp16 = args.opt_level == "O2"
    cfg = TransformerConfig(hidden_size=1024, num_layers=args.layers, num_attention_heads=16, ffn_hidden_size=4096,
                            vocab_size=50304, max_position_embeddings=args.seq, hidden_dropout=args.dropout,
                            attention_dropout=args.dropout, fp16=fp16, bf16=not fp16, masked_softmax_fusion=True,
                            bias_gelu_fusion=True, sequence_parallel=args.sp and tp > 1)
    model = GPTModel(cfg, parallel_output=True).cuda()
    nparams_local = sum(p.numel() for p in model.parameters())
    from beforeholiday_amd.utils import graph_rng

    use_graph = args.graph == "on" or (args.graph == "auto" and world == 1 and args.opt_level == "O5")
    if use_graph:
        graph_rng.enable(seed=rank)  # replayable dropout seeds: a per-call salt + a device step seed
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01, capturable=use_graph)
    model, opt = amp.initialize(model, opt, opt_level=args.opt_level, verbosity=0)
    if dp > 1:
        model = DistributedDataParallel(model, process_group=parallel_state.get_data_parallel_group())

    # every TP rank of one DP replica sees the same tokens
    g = torch.Generator(device="cuda").manual_seed(1000 + parallel_state.get_data_parallel_rank())
    B, S = args.batch, args.seq
    tokens = torch.randint(0, 50257, (B, S), device="cuda", generator=g)
    labels = torch.randint(0, 50257, (B, S), device="cuda", generator=g)
    mask, _, pos = get_ltor_masks_and_position_ids(tokens, -1, False, False, False)

    def step():
        graph_rng.new_step()
        loss = model(tokens, pos, mask, labels=labels).float().mean()
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        if tp > 1:
            finalize_model_grads(getattr(model, "module", model))
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
            print(f"[bench_gpt] {graph_report}", file=sys.stderr, flush=True)
        run()
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
    toks = B * dp * S * args.steps / el
    # 6*N*T matmul FLOPs + causal attention (12*L*h*S per token, halved by the causal skip)
    nparams = 50304 * 1024 + S * 1024 + 2048 + args.layers * 12_596_224  # whole model (355 M at 24 x 1024)
    flops_per_tok = 6 * nparams + 6 * args.layers * 1024 * S
    if rank == 0:
        print(json.dumps({
            "metric": "GPT-2-medium tensor-parallel training tokens/sec", "value": round(toks, 1),
            "unit": "tokens/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
            "model_tflops_per_gpu": round(toks * flops_per_tok / world / 1e12, 1),
            "dtype": "fp16" if fp16 else "bf16", "data": "synthetic token ids, random-init weights",
            "config": {"model": f"GPT-2-medium ({args.layers} layers, {nparams_local / 1e6:.0f}M params per TP rank) "
                       "+ FusedAdam", "global_batch": B * dp, "seq_len": S,
                       "parallelism": f"tp{tp}{'-sp' if cfg.sequence_parallel else ''}-dp{dp}",
                       "final_loss": round(float(loss.detach()), 4)},
            "gemm_table": gemm_tuning.status(), "hip_graph": run is not step,
            "graph_check": graph_report.get("graph")}), flush=True)
    gemm_tuning.finish(args.gemm_table, rank)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
