# round 3: the recomputed BN-backward dgrad on the original epilogue: parity (kernel, layerwise, steps), step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "recompute or bn_backward_fusion or big_tiles or int8" --timeout 300 --timeout-method thread > gpurun_out/r03e_kern_tests.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03e_kern_tests.log; exit 1; }
tail -2 gpurun_out/r03e_kern_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03e_bench_r$i.json 2> gpurun_out/r03e_bench_r$i.err || exit $?
  timeout -k 10 200 env RN_BN_BWD_RECOMPUTE=0 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03e_bench_n$i.json 2> gpurun_out/r03e_bench_n$i.err || exit $?
done
for f in gpurun_out/r03e_bench_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 900 python -u -m pytest tests/test_step_bf16_gpu.py tests/test_step_gpu.py tests/test_int8_gpu.py -x -q -s --timeout 800 --timeout-method thread > gpurun_out/r03e_step.log 2>&1 || { echo "step tests rc=$?"; tail -40 gpurun_out/r03e_step.log; exit 1; }
tail -2 gpurun_out/r03e_step.log
