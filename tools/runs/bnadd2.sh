# fused ReLU-backward + BN reductions of the post-activation tail: kernel tests, whole-step parity, C4 A/B, C4 profile
tools/gpu_steps.sh \
 "200 python -u -m pytest tests/test_kernels_gpu.py -k 'bn_apply_add or relu_bwd_bnred' -x -q --timeout 120 --timeout-method thread > gpurun_out/bb_kern.log 2>&1" \
 "500 python -u -m pytest tests/test_step_gpu.py tests/test_dist_gpu.py tests/test_multidev_gpu.py tests/test_eval_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bb_step.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/bb_c4_on.log 2>&1" \
 "200 env RN_BN_ADD_FUSION=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/bb_c4_off.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/bb_c4_on1.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh bb_c41s --model resnext50 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/bb_c41s_prof.log 2>&1"
