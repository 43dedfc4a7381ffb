# round 3: igemm_big epilogue without block barriers (wave-local LDS waits): conv tests, per-layer A/B, step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_int8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03p_kern.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03p_kern.log; exit 1; }
tail -1 gpurun_out/r03p_kern.log
timeout -k 10 300 python tools/conv_bench.py --only fwd,dgrad > gpurun_out/r03p_cb_new.log 2>&1 || exit $?
timeout -k 10 300 env RN_TUNE=16=1 python tools/conv_bench.py --only fwd,dgrad > gpurun_out/r03p_cb_old.log 2>&1 || exit $?
tail -1 gpurun_out/r03p_cb_new.log gpurun_out/r03p_cb_old.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03p_c2_f$i.json 2> gpurun_out/r03p_c2_f$i.err || exit $?
  timeout -k 10 200 env RN_TUNE=16=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03p_c2_n$i.json 2> gpurun_out/r03p_c2_n$i.err || exit $?
done
for f in gpurun_out/r03p_c2_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
