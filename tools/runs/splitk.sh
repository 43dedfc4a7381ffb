# FC forward split-K: golden / kernel / step tests, bench, one-stream profile
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_golden_gpu.py tests/test_kernels_gpu.py tests/test_step_gpu.py tests/test_step_bf16_gpu.py tests/test_eval_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sk_test.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/sk_bench.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh sk1s --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/sk1s_prof.log 2>&1"
