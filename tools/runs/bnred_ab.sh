# conflict-free BN block reductions: BN kernel tests + golden, step parity, bench A/B vs the previous commit's library
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py tests/test_golden_gpu.py -k 'bn or relu_bwd' -x -q --timeout 120 --timeout-method thread > gpurun_out/br_kern.log 2>&1" \
 "300 python -u -m pytest tests/test_step_gpu.py tests/test_step_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/br_step.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/br_bench0.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh br1s --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/br1s_prof.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/br_bench1.log 2>&1"
