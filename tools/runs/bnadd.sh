# BN-apply + add fusion (post-activation units): kernel bit-exactness, whole-step parity, C4 / C1 bench, C4 profile
tools/gpu_steps.sh \
 "200 python -u -m pytest tests/test_kernels_gpu.py -k 'bn_apply_add' -x -q --timeout 120 --timeout-method thread > gpurun_out/ba_kern.log 2>&1" \
 "500 python -u -m pytest tests/test_step_gpu.py tests/test_step_bf16_gpu.py tests/test_eval_gpu.py tests/test_graph_passes_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_step.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/ba_c4_on.log 2>&1" \
 "200 env RN_BN_ADD_FUSION=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/ba_c4_off.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh ba_c41s --model resnext50 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/ba_c41s_prof.log 2>&1"
