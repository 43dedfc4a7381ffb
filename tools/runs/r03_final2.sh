# round-3 closing run after the BatchNorm cache hints (rn_set_tuning 18 = 7): full GPU suite, smoke,
# default bench line, rocprofv3 kernel trace of the bench, PMC passes, C4 / C5 bench lines
tools/gpu_steps.sh \
 "600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h_gputest.log 2>&1" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r03h_smoke.log 2>&1" \
 "300 python bench.py > gpurun_out/r03h_bench.log 2>&1" \
 "240 bash tools/prof_bench.sh r03h --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03h_prof.log 2>&1" \
 "900 bash tools/pmc_bench.sh r03h --steps 3 --warmup 1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03h_pmc.log 2>&1" \
 "150 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03h_c4.log 2>&1" \
 "150 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03h_c5.log 2>&1"
tail -n2 gpurun_out/r03h_gputest.log; tail -n1 gpurun_out/r03h_smoke.log; tail -n1 gpurun_out/r03h_bench.log | cut -c1-300
