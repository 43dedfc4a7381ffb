# debug: test_dgrad_bn_backward_fusion with the current build and with the last commit's build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "bn_backward_fusion and auto and rows224 and case0" --timeout 120 --timeout-method thread > gpurun_out/r03i_cur.log 2>&1; echo "current rc=$?"
timeout -k 10 300 env RN_LIB_PATH=$PWD/oldlib_tmp/librn_prev.so python -u -m pytest tests/test_kernels_gpu.py -x -q -k "bn_backward_fusion and auto and rows224 and case0" --timeout 120 --timeout-method thread > gpurun_out/r03i_prev.log 2>&1; echo "prev rc=$?"
tail -3 gpurun_out/r03i_cur.log gpurun_out/r03i_prev.log
