# BN partials combined per tile: kernel tests (bnstats / dgrad fusion / int8 / tiles), whole-step parity, bench, one-stream profile
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_kernels_gpu.py tests/test_int8_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pr_kern.log 2>&1" \
 "500 python -u -m pytest tests/test_step_gpu.py tests/test_step_bf16_gpu.py tests/test_graph_passes_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pr_step.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/pr_bench0.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/pr_bench1.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh pr1s --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/pr1s_prof.log 2>&1"
