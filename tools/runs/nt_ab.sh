# BatchNorm apply passes with nontemporal stores / loads (rn_set_tuning 18): full GPU suite, smoke,
# then C2 bench pairs default / 18=1 / 18=3 interleaved on one box
B="python bench.py --no-cpu-baseline --pcie-steps 0"
tools/gpu_steps.sh \
 "420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nt/gputest.log 2>&1" \
 "120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/nt/smoke.log 2>&1" \
 "120 $B > gpurun_out/nt/c2_n1.json 2>gpurun_out/nt/err.log" \
 "120 env RN_TUNE=18=1 $B > gpurun_out/nt/c2_s1.json 2>>gpurun_out/nt/err.log" \
 "120 env RN_TUNE=18=3 $B > gpurun_out/nt/c2_b1.json 2>>gpurun_out/nt/err.log" \
 "120 $B > gpurun_out/nt/c2_n2.json 2>>gpurun_out/nt/err.log" \
 "120 env RN_TUNE=18=1 $B > gpurun_out/nt/c2_s2.json 2>>gpurun_out/nt/err.log" \
 "120 env RN_TUNE=18=3 $B > gpurun_out/nt/c2_b2.json 2>>gpurun_out/nt/err.log"
