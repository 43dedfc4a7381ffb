# round-2 last check after the grouped weight-gradient split sizing: full GPU suite and smoke
tools/gpu_steps.sh \
 "600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f5_gputest.log 2>&1" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/f5_smoke.log 2>&1"
