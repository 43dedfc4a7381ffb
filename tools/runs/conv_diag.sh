# per-layer conv times with the igemm_big_kernel schedule diagnostics (rn_set_tuning 7 bits):
# 16 = no epilogue, 8 = no DMAs in the main loop, 4 = no waits / barriers (wrong results; timing only)
for v in 0 16 8 4 28; do
  timeout -k 10 120 env RN_TUNE="7=$v" python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/cdiag_$v.log 2>&1 || exit $?
done
