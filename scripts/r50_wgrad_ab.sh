# same-box A/B of the headline step: MFMA conv wgrad (auto) vs MIOpen wgrad, alternating
for i in 1 2; do
  for v in auto miopen; do
    if [ $v = miopen ]; then export BH_CONV_WGRAD=miopen; else unset BH_CONV_WGRAD; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_$v$i.log 2>&1 || exit 1
    echo "$v $i: $(tail -1 gpurun_out/ab_$v$i.log | cut -c1-130)"
  done
done
