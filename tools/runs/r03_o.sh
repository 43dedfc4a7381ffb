# round 3 checkpoint: full GPU suite, smoke, headline bench, C4 / C5 bench lines
tools/gpu_steps.sh \
 "900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03o_gputest.log 2>&1" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r03o_smoke.log 2>&1" \
 "300 python bench.py > gpurun_out/r03o_bench.log 2>&1" \
 "150 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03o_c4.log 2>&1" \
 "150 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03o_c5.log 2>&1"
tail -3 gpurun_out/r03o_gputest.log; tail -2 gpurun_out/r03o_smoke.log; tail -1 gpurun_out/r03o_bench.log | cut -c1-400; tail -1 gpurun_out/r03o_c4.log | cut -c1-200; tail -1 gpurun_out/r03o_c5.log | cut -c1-200
