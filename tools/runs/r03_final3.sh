# round-3 final check on the final HEAD (rn_set_tuning 18 = 23: conv tile outputs with the streaming
# hint too): full GPU suite, smoke, default bench line, C4 / C5 bench lines
tools/gpu_steps.sh \
 "600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03i_gputest.log 2>&1" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r03i_smoke.log 2>&1" \
 "300 python bench.py > gpurun_out/r03i_bench.log 2>&1" \
 "120 env RN_TUNE=18=7 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03i_c2_7.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03i_c2_23.log 2>&1" \
 "150 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03i_c4.log 2>&1" \
 "150 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03i_c5.log 2>&1"
tail -n2 gpurun_out/r03i_gputest.log; tail -n1 gpurun_out/r03i_smoke.log; tail -n1 gpurun_out/r03i_bench.log | cut -c1-300
