# round 3: deterministic weight gradients (tests), kernel + step parity after the wgrad epilogue change,
# PIPE (non-XF 224x256 tiles) step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_deterministic_gpu.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/r03f_det.log 2>&1 || { echo "det tests rc=$?"; tail -40 gpurun_out/r03f_det.log; exit 1; }
grep -E "PASSED|FAILED|ReLU|gradient error|probabilities" gpurun_out/r03f_det.log | tail -20
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_int8_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f_kern.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03f_kern.log; exit 1; }
tail -1 gpurun_out/r03f_kern.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03f_bench_a$i.json 2> gpurun_out/r03f_bench_a$i.err || exit $?
  timeout -k 10 200 env RN_TUNE=16=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03f_bench_p$i.json 2> gpurun_out/r03f_bench_p$i.err || exit $?
done
for f in gpurun_out/r03f_bench_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 900 python -u -m pytest tests/test_step_gpu.py tests/test_step_bf16_gpu.py -x -q -s --timeout 800 --timeout-method thread > gpurun_out/r03f_step.log 2>&1 || { echo "step tests rc=$?"; tail -40 gpurun_out/r03f_step.log; exit 1; }
tail -1 gpurun_out/r03f_step.log
