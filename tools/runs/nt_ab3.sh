# rn_set_tuning 18 default 15 (hints in the reduction / residual-tail passes and the int8 quantizer
# pass too): full GPU suite, smoke, then bench pairs 15 (default) vs 3 on C2 / C4, and 15 / 7 / 3 on C5
B="python bench.py --no-cpu-baseline --pcie-steps 0"
O=gpurun_out/nt3
tools/gpu_steps.sh \
 "420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1" \
 "120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "120 $B > $O/c2_d1.json 2>$O/err.log" \
 "120 env RN_TUNE=18=3 $B > $O/c2_a1.json 2>>$O/err.log" \
 "120 $B > $O/c2_d2.json 2>>$O/err.log" \
 "120 env RN_TUNE=18=3 $B > $O/c2_a2.json 2>>$O/err.log" \
 "150 $B --model resnext50 > $O/c4_d1.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=3 $B --model resnext50 > $O/c4_a1.json 2>>$O/err.log" \
 "150 $B --model resnext50 > $O/c4_d2.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=3 $B --model resnext50 > $O/c4_a2.json 2>>$O/err.log" \
 "150 $B --model resnet50_int8 > $O/c5_d1.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=7 $B --model resnet50_int8 > $O/c5_r1.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=3 $B --model resnet50_int8 > $O/c5_a1.json 2>>$O/err.log" \
 "150 $B --model resnet50_int8 > $O/c5_d2.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=7 $B --model resnet50_int8 > $O/c5_r2.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=3 $B --model resnet50_int8 > $O/c5_a2.json 2>>$O/err.log"
