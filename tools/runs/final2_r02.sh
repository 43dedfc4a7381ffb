# round-2 closing check after the grouped zero-block skips: full GPU suite, smoke, headline bench x2, C4 bench
tools/gpu_steps.sh \
 "600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f2_gputest.log 2>&1" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/f2_smoke.log 2>&1" \
 "300 python bench.py > gpurun_out/f2_bench.log 2>&1" \
 "150 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/f2_bench2.log 2>&1" \
 "150 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/f2_c4.log 2>&1"
