# 64-output-channel 3x3 layers on the 224x128 tile (rn_set_tuning 4 = 6) vs the 256x64 tile: per-layer conv_bench + bench pair
tools/gpu_steps.sh \
 "120 python tools/conv_bench.py --only fwd,dgrad --filter stage1_unit1_conv2 --iters 20 > gpurun_out/k64_cb_def.log 2>&1" \
 "120 env RN_TUNE=4=6 python tools/conv_bench.py --only fwd,dgrad --filter stage1_unit1_conv2 --iters 20 > gpurun_out/k64_cb_6.log 2>&1" \
 "200 env RN_TUNE=4=6 python -u -m pytest tests/test_step_gpu.py -x -q -k resnet50 --timeout 200 --timeout-method thread > gpurun_out/k64_step.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/k64_def.log 2>&1" \
 "120 env RN_TUNE=4=6 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/k64_6.log 2>&1"
