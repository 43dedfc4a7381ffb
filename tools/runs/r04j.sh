# weight-gradient split at 50 % by default: the GPU suite, then a finer sweep of rn_set_tuning 21 (C2 pairs, C4, C5)
tools/gpu_steps.sh \
 "900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04j_gputest.log 2>&1" \
 "200 env RN_TUNE=21=40 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c2_40.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c2_50.log 2>&1" \
 "200 env RN_TUNE=21=60 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c2_60.log 2>&1" \
 "200 env RN_TUNE=21=33 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c2_33.log 2>&1" \
 "200 env RN_TUNE=21=40 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c2_40b.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c2_50b.log 2>&1" \
 "200 env RN_TUNE=21=60 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c2_60b.log 2>&1" \
 "200 env RN_TUNE=21=40 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c4_40.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c4_50.log 2>&1" \
 "200 env RN_TUNE=21=40 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c5_40.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04j_c5_50.log 2>&1"
tail -n2 gpurun_out/r04j_gputest.log
for f in c2_40 c2_50 c2_60 c2_33 c2_40b c2_50b c2_60b c4_40 c4_50 c5_40 c5_50; do echo -n "$f "; tail -n1 gpurun_out/r04j_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
