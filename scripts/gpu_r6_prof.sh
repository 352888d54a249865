#!/bin/bash
# round-6 profiles: ResNet-50 kernel summary, ResNet-50 PMC passes (conv / GEMM families), BERT-large summary
bash scripts/prof_resnet.sh || exit $?
echo "resnet summary: $(head -3 gpurun_out/resnet_summary.md | tail -1)"
bash scripts/pmc_resnet.sh || exit $?
bash scripts/prof_bert.sh || exit $?
echo "bert summary: $(head -3 gpurun_out/bert_summary.md | tail -1)"
