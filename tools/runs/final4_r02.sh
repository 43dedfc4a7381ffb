# round-2 closing check (grouped wgrad blocks over four waves): full GPU suite, smoke,
# headline bench, rocprofv3 trace of the bench step, C4 bench
tools/gpu_steps.sh \
 "600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f4_gputest.log 2>&1" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/f4_smoke.log 2>&1" \
 "300 python bench.py > gpurun_out/f4_bench.log 2>&1" \
 "240 bash tools/prof_bench.sh r02h --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r02h_prof.log 2>&1" \
 "150 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/f4_c4.log 2>&1"
