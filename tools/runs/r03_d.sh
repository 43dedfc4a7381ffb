# round 3: transposed-accumulator bf16 epilogue (all igemm_big variants), PIPE, the recomputed
# BN-backward dgrad: kernel parity, conv timing, step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_int8_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d_kern_tests.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/r03d_kern_tests.log; exit 1; }
tail -2 gpurun_out/r03d_kern_tests.log
timeout -k 10 150 python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/r03d_cb_tr.log 2>&1 || exit $?
timeout -k 10 150 env RN_TUNE=16=1 python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/r03d_cb_tr_pipe.log 2>&1 || exit $?
grep per-step gpurun_out/r03d_cb_tr.log gpurun_out/r03d_cb_tr_pipe.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03d_bench_a$i.json 2> gpurun_out/r03d_bench_a$i.err || exit $?
  timeout -k 10 200 env RN_TUNE=16=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03d_bench_p$i.json 2> gpurun_out/r03d_bench_p$i.err || exit $?
  timeout -k 10 200 env RN_BN_BWD_RECOMPUTE=0 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03d_bench_n$i.json 2> gpurun_out/r03d_bench_n$i.err || exit $?
done
for f in gpurun_out/r03d_bench_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 900 python -u -m pytest tests/test_step_bf16_gpu.py tests/test_step_gpu.py -x -q --timeout 800 --timeout-method thread > gpurun_out/r03d_step.log 2>&1 || { echo "step tests rc=$?"; tail -40 gpurun_out/r03d_step.log; exit 1; }
tail -2 gpurun_out/r03d_step.log
