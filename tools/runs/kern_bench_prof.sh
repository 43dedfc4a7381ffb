# kernel parity subset, whole-step parity, bench, one-stream rocprof trace (per-layer table)
tag=${1:-x4}
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -k 'bnrelu or wgrad or conv_fwd' -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_kern.log 2>&1" \
 "300 python -u -m pytest tests/test_step_bf16_gpu.py tests/test_step_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_step.log 2>&1" \
 "150 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_bench.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh ${tag}1s --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}1s_prof.log 2>&1"
