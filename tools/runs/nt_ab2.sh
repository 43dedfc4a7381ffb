# rn_set_tuning 18 default 3 (nontemporal loads + stores in the BatchNorm apply passes): full GPU
# suite, smoke, then C2 / C4 / C5 bench pairs 3 (default) / 7 (read passes too) / 0 (no hints)
B="python bench.py --no-cpu-baseline --pcie-steps 0"
O=gpurun_out/nt2
tools/gpu_steps.sh \
 "420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1" \
 "120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "120 $B > $O/c2_d1.json 2>$O/err.log" \
 "120 env RN_TUNE=18=7 $B > $O/c2_r1.json 2>>$O/err.log" \
 "120 env RN_TUNE=18=0 $B > $O/c2_z1.json 2>>$O/err.log" \
 "120 $B > $O/c2_d2.json 2>>$O/err.log" \
 "120 env RN_TUNE=18=7 $B > $O/c2_r2.json 2>>$O/err.log" \
 "120 env RN_TUNE=18=0 $B > $O/c2_z2.json 2>>$O/err.log" \
 "150 $B --model resnext50 > $O/c4_d1.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=7 $B --model resnext50 > $O/c4_r1.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=0 $B --model resnext50 > $O/c4_z1.json 2>>$O/err.log" \
 "150 $B --model resnet50_int8 > $O/c5_d1.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=7 $B --model resnet50_int8 > $O/c5_r1.json 2>>$O/err.log" \
 "150 env RN_TUNE=18=0 $B --model resnet50_int8 > $O/c5_z1.json 2>>$O/err.log"
