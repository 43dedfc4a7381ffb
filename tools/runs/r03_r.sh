# round 3: the quantizers' max from the int8 conv epilogue's per-block extremes (rn_conv_fwd_i8_mm): parity + C5 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_int8_gpu.py tests/test_kernels_gpu.py -k "stem or int8 or quant" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03r_kern.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03r_kern.log; exit 1; }
tail -1 gpurun_out/r03r_kern.log
timeout -k 10 900 python -u -m pytest tests/test_step_gpu.py tests/test_graph_passes_gpu.py -x -q -s -k "int8 or quant" --timeout 800 --timeout-method thread > gpurun_out/r03r_step.log 2>&1 || { echo "step tests rc=$?"; tail -40 gpurun_out/r03r_step.log; exit 1; }
tail -1 gpurun_out/r03r_step.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03r_c5_f$i.json 2> gpurun_out/r03r_c5_f$i.err || exit $?
  timeout -k 10 200 env RN_QUANT_BN_MM=0 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03r_c5_n$i.json 2> gpurun_out/r03r_c5_n$i.err || exit $?
done
for f in gpurun_out/r03r_c5_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 240 bash tools/prof_bench.sh r03r_c5 --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03r_prof.log 2>&1 || exit $?
python3 tools/step_breakdown.py gpurun_out/prof_r03r_c5/run_kernel_trace.csv > gpurun_out/r03r_breakdown.txt && head -30 gpurun_out/r03r_breakdown.txt
