# end-of-session validation: full GPU suite, smoke, headline bench (what the driver runs at round end)
bash scripts/gpu_steps.sh \
 "gputests:1000:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:400:python bench.py --steps 20 --warmup 5"
