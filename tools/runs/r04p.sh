# closing checks on the new defaults: the GPU suite, smoke, the default bench line
tools/gpu_steps.sh \
 "900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04p_gputest.log 2>&1" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04p_smoke.log 2>&1" \
 "400 python bench.py > gpurun_out/r04p_bench.log 2>&1"
tail -n2 gpurun_out/r04p_gputest.log; tail -n1 gpurun_out/r04p_bench.log
