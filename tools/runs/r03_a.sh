# round 3, first GPU call: bench --gpus 2 launch test, epoch-end aux/resume test, the bf16 full-size
# parity numbers (-s), and a baseline bench line on this box
tools/gpu_steps.sh \
 "500 python -u -m pytest tests/test_bench_launch.py tests/test_epoch_end_gpu.py -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1" \
 "500 python -u -m pytest tests/test_step_bf16_gpu.py -k full_size_gradients -x -v -s --timeout 450 --timeout-method thread > gpurun_out/r03a_bf16full.log 2>&1" \
 "300 python bench.py > gpurun_out/r03a_bench.log 2>&1"
