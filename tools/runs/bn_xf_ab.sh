tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -k bnrelu_on_load -x -q --timeout 120 --timeout-method thread > gpurun_out/x1_kern.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/x1_bench_a0.log 2>&1" \
 "120 env RN_BN_APPLY_FUSION=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/x1_bench_b0.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/x1_bench_a1.log 2>&1" \
 "120 env RN_BN_APPLY_FUSION=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/x1_bench_b1.log 2>&1" \
 "400 env RN_BN_APPLY_FUSION=1 python -u -m pytest tests/test_step_bf16_gpu.py tests/test_step_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/x1_step.log 2>&1"
