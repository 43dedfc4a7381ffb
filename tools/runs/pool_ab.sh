# 2x2-block max-pool backward: kernel tests, step parity, bench pair, one-stream profile
tools/gpu_steps.sh \
 "200 python -u -m pytest tests/test_kernels_gpu.py -k 'maxpool' tests/test_golden_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pl_kern.log 2>&1" \
 "300 python -u -m pytest tests/test_step_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pl_step.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/pl_on.log 2>&1" \
 "120 env RN_TUNE=12=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/pl_off.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh pl1s --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/pl1s_prof.log 2>&1"
