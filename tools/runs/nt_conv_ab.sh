# conv tile epilogue stores with the nontemporal hint (rn_set_tuning 18 bit 16, opt-in): conv kernel
# tests and a ResNet-50 step test with the bit set, then C2 / C4 bench pairs 7 (default) vs 23
B="python bench.py --no-cpu-baseline --pcie-steps 0"
O=gpurun_out/ntc
tools/gpu_steps.sh \
 "300 env RN_TUNE=18=23 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_bf16_gpu.py -k 'conv or bnstats or bnred or step' -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1" \
 "120 $B > $O/c2_d1.json 2>$O/err.log" \
 "120 env RN_TUNE=18=23 $B > $O/c2_c1.json 2>>$O/err.log" \
 "120 $B > $O/c2_d2.json 2>>$O/err.log" \
 "120 env RN_TUNE=18=23 $B > $O/c2_c2.json 2>>$O/err.log" \
 "150 $B --model resnext50 > $O/c4_d1.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=23 $B --model resnext50 > $O/c4_c1.json 2>>$O/err.log"
