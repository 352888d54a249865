# BERT-large O2 + FusedLAMB and GPT-2-medium with the latest kernels; BERT with host vs device loss scaler
bash scripts/gpu_steps.sh \
 "bert_host:400:python benchmarks/bench_bert.py --steps 10 --warmup 3" \
 "bert_dev:400:BH_AMP_DEVICE_SCALER=1 python benchmarks/bench_bert.py --steps 10 --warmup 3" \
 "gpt:400:python benchmarks/bench_gpt.py"
