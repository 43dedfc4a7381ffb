# round 3: the stem's quantizer clip gradient with LDS weights and a 16-byte scan: parity + C5 step
# parity + C5 step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_int8_gpu.py tests/test_kernels_gpu.py -k "stem or int8 or quant" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03l_kern.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03l_kern.log; exit 1; }
tail -1 gpurun_out/r03l_kern.log
timeout -k 10 900 python -u -m pytest tests/test_step_gpu.py tests/test_graph_passes_gpu.py -x -q -s -k "int8 or quant" --timeout 800 --timeout-method thread > gpurun_out/r03l_step.log 2>&1 || { echo "step tests rc=$?"; tail -40 gpurun_out/r03l_step.log; exit 1; }
tail -1 gpurun_out/r03l_step.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03l_c5_f$i.json 2> gpurun_out/r03l_c5_f$i.err || exit $?
done
for f in gpurun_out/r03l_c5_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 240 bash tools/prof_bench.sh r03l_c5 --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03l_prof.log 2>&1 || exit $?
tail -3 gpurun_out/r03l_prof.log
