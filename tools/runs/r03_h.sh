# round 3: the int8 graph's quantizer STE folded into the BN backward: parity + C5 step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_int8_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h_kern.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03h_kern.log; exit 1; }
tail -1 gpurun_out/r03h_kern.log
timeout -k 10 900 python -u -m pytest tests/test_step_gpu.py tests/test_graph_passes_gpu.py -x -q -s --timeout 800 --timeout-method thread > gpurun_out/r03h_step.log 2>&1 || { echo "step tests rc=$?"; tail -40 gpurun_out/r03h_step.log; exit 1; }
tail -1 gpurun_out/r03h_step.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03h_c5_f$i.json 2> gpurun_out/r03h_c5_f$i.err || exit $?
  timeout -k 10 200 env RN_QUANT_BWD_FOLD=0 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03h_c5_n$i.json 2> gpurun_out/r03h_c5_n$i.err || exit $?
done
for f in gpurun_out/r03h_c5_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03h_c2.json 2> gpurun_out/r03h_c2.err || exit $?
python3 -c "import json,sys; d=json.loads(open('gpurun_out/r03h_c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'])"
