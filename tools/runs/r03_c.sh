# round 3: W1S (4 waves, one per SIMD) and PIPE (main loop pipelined across the barrier) 224x256 tile
# variants vs the 8-wave tile; parity of the new variants; conv schedule diagnostics per layer
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "w1s or pipe" --timeout 120 --timeout-method thread > gpurun_out/r03c_new_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r03c_new_tests.log; exit 1; }
tail -3 gpurun_out/r03c_new_tests.log
timeout -k 10 150 python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/r03c_cb_base.log 2>&1 || exit $?
timeout -k 10 150 env RN_TUNE=16=1 python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/r03c_cb_pipe.log 2>&1 || exit $?
timeout -k 10 150 env RN_TUNE=15=2 python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/r03c_cb_w1s.log 2>&1 || exit $?
for v in 16 8 4 28; do
  timeout -k 10 150 env RN_DIAG=1 RN_TUNE="7=$v" python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/r03c_cdiag_$v.log 2>&1 || exit $?
done
tail -2 gpurun_out/r03c_cb_*.log gpurun_out/r03c_cdiag_*.log
