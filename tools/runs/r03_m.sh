# round 3: stem clip-gradient gathers (scalar index math, all taps in flight) and the batched weight
# quantization (rn_weight_quant_pack): parity + C5 step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/probe/stem_clip_probe.py > gpurun_out/r03m_stem_probe.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/r03m_stem_probe.log; exit 1; }
cat gpurun_out/r03m_stem_probe.log
timeout -k 10 400 python -u -m pytest tests/test_int8_gpu.py tests/test_kernels_gpu.py -k "stem or int8 or quant" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03m_kern.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03m_kern.log; exit 1; }
tail -1 gpurun_out/r03m_kern.log
timeout -k 10 900 python -u -m pytest tests/test_step_gpu.py tests/test_graph_passes_gpu.py -x -q -s -k "int8 or quant" --timeout 800 --timeout-method thread > gpurun_out/r03m_step.log 2>&1 || { echo "step tests rc=$?"; tail -40 gpurun_out/r03m_step.log; exit 1; }
tail -1 gpurun_out/r03m_step.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03m_c5_f$i.json 2> gpurun_out/r03m_c5_f$i.err || exit $?
  timeout -k 10 200 env RN_WQUANT_BATCH=0 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03m_c5_n$i.json 2> gpurun_out/r03m_c5_n$i.err || exit $?
done
for f in gpurun_out/r03m_c5_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 240 bash tools/prof_bench.sh r03m_c5 --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03m_prof.log 2>&1 || exit $?
python3 tools/step_breakdown.py gpurun_out/prof_r03m_c5/run_kernel_trace.csv > gpurun_out/r03m_breakdown.txt && head -30 gpurun_out/r03m_breakdown.txt
