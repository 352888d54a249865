# flash attention counters at the GPT shape (dropout 0.1) and BERT shape (no dropout)
bash scripts/gpu_steps.sh \
 "pmc_gpt:400:bash scripts/pmc_flash.sh --shape gpt --dropout 0.1 && mv gpurun_out/pmcf gpurun_out/pmcf_gpt" \
 "pmc_bert:400:bash scripts/pmc_flash.sh --shape bert --dropout 0"
