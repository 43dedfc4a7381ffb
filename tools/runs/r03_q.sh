# round 3: direct grouped weight gradient (4 per group): parity, per-layer timing, C4 step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "grouped" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03q_kern.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03q_kern.log; exit 1; }
tail -1 gpurun_out/r03q_kern.log
timeout -k 10 300 python tools/conv_bench.py --graph resnext50 --filter conv2 > gpurun_out/r03q_cb.log 2>&1 || { echo "conv bench rc=$?"; tail -20 gpurun_out/r03q_cb.log; exit 1; }
cat gpurun_out/r03q_cb.log
timeout -k 10 900 python -u -m pytest tests/ -x -q -s -k "resnext" -m gpu --timeout 800 --timeout-method thread > gpurun_out/r03q_step.log 2>&1 || { echo "step tests rc=$?"; tail -40 gpurun_out/r03q_step.log; exit 1; }
tail -1 gpurun_out/r03q_step.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03q_c4_f$i.json 2> gpurun_out/r03q_c4_f$i.err || exit $?
  timeout -k 10 200 env RN_TUNE=15=1 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03q_c4_n$i.json 2> gpurun_out/r03q_c4_n$i.err || exit $?
done
for f in gpurun_out/r03q_c4_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
