# Round 2 GPU pass B: full GPU suite after the contrib/optimizer/transducer/amp-RNN additions.
bash scripts/gpu_steps.sh \
 "gputests:700:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'"
