# W4 tile: kernel parity (forced on every 1x1 pad-0 conv), whole-step bf16 parity, bench A/B (on / off)
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_kernels_gpu.py -k 'bnstats or dgrad_bn or bnrelu_on_load_tiles or big_tiles' -x -q --timeout 120 --timeout-method thread > gpurun_out/w4_kern.log 2>&1" \
 "400 python -u -m pytest tests/test_step_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w4_step.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/w4_b_on0.log 2>&1" \
 "120 env RN_TUNE=11=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/w4_b_off0.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/w4_b_on1.log 2>&1" \
 "120 env RN_TUNE=11=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/w4_b_off1.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh w41s --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/w41s_prof.log 2>&1"
