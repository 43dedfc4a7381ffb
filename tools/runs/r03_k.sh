# round 3: the two quantizers of a stage's first unit: one fused forward call, folded into the BN backward:
# parity + C5 step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_int8_gpu.py tests/test_kernels_gpu.py -k "int8 or quant or bn_backward or bn_" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03k_kern.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03k_kern.log; exit 1; }
tail -1 gpurun_out/r03k_kern.log
timeout -k 10 900 python -u -m pytest tests/test_step_gpu.py tests/test_graph_passes_gpu.py -x -q -s -k "int8 or quant" --timeout 800 --timeout-method thread > gpurun_out/r03k_step.log 2>&1 || { echo "step tests rc=$?"; tail -40 gpurun_out/r03k_step.log; exit 1; }
tail -1 gpurun_out/r03k_step.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03k_c5_f$i.json 2> gpurun_out/r03k_c5_f$i.err || exit $?
  timeout -k 10 200 env RN_QUANT_BWD_FOLD=0 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03k_c5_n$i.json 2> gpurun_out/r03k_c5_n$i.err || exit $?
done
for f in gpurun_out/r03k_c5_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 240 bash tools/prof_bench.sh r03k_c5 --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03k_prof.log 2>&1 || exit $?
tail -3 gpurun_out/r03k_prof.log
