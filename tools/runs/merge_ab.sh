# one-launch BN merge + finalize: kernel tests, whole-step parity, bench A/B (rn_set_tuning 12)
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -k 'bn_part_merge or bnstats' -x -q --timeout 120 --timeout-method thread > gpurun_out/mg_kern.log 2>&1" \
 "400 python -u -m pytest tests/test_step_gpu.py tests/test_step_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mg_step.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/mg_on0.log 2>&1" \
 "120 env RN_TUNE=12=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/mg_off0.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/mg_on1.log 2>&1" \
 "120 env RN_TUNE=12=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/mg_off1.log 2>&1"
