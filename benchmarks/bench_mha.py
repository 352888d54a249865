"""Self-attention block ms/layer at the reference's only published shapes.

Published numbers: apex/contrib/multihead_attn/README.md:54-60 + MHA_fwd.png / MHA_bwd.png (Titan V,
hidden 1024, 16 heads, seq 64, dropout 0.1, fp16, no biases; harness defaults
apex/contrib/examples/multihead_attn/perf_test_multihead_attn.py:9-23: 18 layers chained, 20 timed
trials after 5 warmup, fwd / bwd timed with events around the whole chain, reported per layer).
Values below are read off the charts (±0.02 ms). We time our ``impl='fast'`` block, our
``impl='default'`` block and ``torch.nn.MultiheadAttention`` the same way and print one JSON line
per (impl, tokens) with ``vs_published`` = published_ms / our_ms (>1 = faster than the reference).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# tokens: (fwd C++, fwd Python, fwd torch.nn, bwd C++, bwd Python, bwd torch.nn) on Titan V
PUBLISHED = {
    640: (0.20, 0.63, 0.90, 0.32, 0.89, 0.83),
    1280: (0.20, 0.69, 0.87, 0.42, 0.99, 0.83),
    2560: (0.34, 0.66, 0.87, 0.76, 1.03, 0.92),
    3840: (0.55, 0.57, 0.89, 1.04, 1.10, 1.28),
    5120: (0.68, 0.70, 1.06, 1.31, 1.38, 1.69),
    6400: (0.90, 0.91, 1.33, 1.68, 1.76, 2.26),
    7680: (1.02, 1.03, 1.52, 1.95, 2.03, 2.69),
}


def build(impl, layers, hidden, heads):
    from beforeholiday_amd.contrib.multihead_attn import SelfMultiheadAttn

    out = []
    for _ in range(layers):
        if impl == "torch":
            m = torch.nn.MultiheadAttention(hidden, heads, dropout=0.1, bias=False)
        else:
            m = SelfMultiheadAttn(hidden, heads, dropout=0.1, bias=False, impl=impl)
            m.reset_parameters()
        out.append(m.cuda().half())
    return out


def run(layers_mods, impl, seqs, seq_len, hidden, trials, warmup):
    x = torch.randn(seq_len, seqs, hidden, dtype=torch.float16, device="cuda", requires_grad=True)
    g = torch.randn_like(x)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(trials)]
    for t in range(trials + warmup):
        h = x
        e = ev[t - warmup] if t >= warmup else None
        if e:
            e[0].record()
        for m in layers_mods:
            if impl == "torch":
                h, _ = m(h, h, h, need_weights=False)
            else:
                h, _ = m(h, h, h, key_padding_mask=None, need_weights=False, attn_mask=None, is_training=True)
        if e:
            e[1].record()
        h.backward(g)
        if e:
            e[2].record()
    torch.cuda.synchronize()
    fwd = sum(e[0].elapsed_time(e[1]) for e in ev) / (trials * len(layers_mods))
    bwd = sum(e[1].elapsed_time(e[2]) for e in ev) / (trials * len(layers_mods))
    return fwd, bwd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq-length", type=int, default=64)
    ap.add_argument("--hidden-dim", type=int, default=1024)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--layers", type=int, default=18)
    ap.add_argument("--trials", type=int, default=20)
    ap.add_argument("--warmup-trials", type=int, default=5)
    ap.add_argument("--impls", default="fast,default,torch")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from beforeholiday_amd._native import require_native

    require_native("bench_mha")
    torch.manual_seed(111)
    col = {"fast": (0, 3), "default": (1, 4), "torch": (2, 5)}
    rows = []
    for impl in args.impls.split(","):
        mods = build(impl, args.layers, args.hidden_dim, args.heads)
        for tokens in sorted(PUBLISHED):
            seqs = tokens // args.seq_length
            fwd, bwd = run(mods, impl, seqs, args.seq_length, args.hidden_dim, args.trials, args.warmup_trials)
            pf, pb = PUBLISHED[tokens][col[impl][0]], PUBLISHED[tokens][col[impl][1]]
            r = {"bench": "self_attn_ms_per_layer", "impl": impl, "tokens": tokens, "seqs": seqs,
                 "seq_len": args.seq_length, "hidden": args.hidden_dim, "heads": args.heads,
                 "fwd_ms": round(fwd, 4), "bwd_ms": round(bwd, 4),
                 "published_titanv_fwd_ms": pf, "published_titanv_bwd_ms": pb,
                 "vs_published_fwd": round(pf / fwd, 2), "vs_published_bwd": round(pb / bwd, 2)}
            rows.append(r)
            print(json.dumps(r), flush=True)
        del mods
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
