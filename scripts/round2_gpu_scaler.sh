# device-resident loss scaler: GPU tests, same-box A/B of the headline step, kernel-trace idle gaps
bash scripts/gpu_steps.sh \
 "tscaler:300:python -u -m pytest tests/test_amp_device_scaler.py tests/test_amp.py tests/test_l1_cross_product.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "b_dev1:300:python bench.py --steps 30 --warmup 5" \
 "b_host1:300:python bench.py --steps 30 --warmup 5 --host-scaler" \
 "b_dev2:300:python bench.py --steps 30 --warmup 5" \
 "b_host2:300:python bench.py --steps 30 --warmup 5 --host-scaler" \
 "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 5 && python scripts/prof_summary.py gpurun_out/prof_r50 k_lamb2 3 gpurun_out/r50_summary.md && rm -rf gpurun_out/prof_r50"
