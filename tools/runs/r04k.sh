# C4: the grouped band weight gradients' own split percent (rn_set_tuning 23) vs the global one (21)
tools/gpu_steps.sh \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04k_c4_50.log 2>&1" \
 "200 env RN_TUNE=23=40 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04k_c4_g40.log 2>&1" \
 "200 env RN_TUNE=21=40 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04k_c4_40.log 2>&1" \
 "200 env RN_TUNE=23=33 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04k_c4_g33.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04k_c4_50b.log 2>&1" \
 "200 env RN_TUNE=23=40 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04k_c4_g40b.log 2>&1" \
 "200 env RN_TUNE=21=40 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04k_c4_40b.log 2>&1" \
 "200 env RN_TUNE=21=40,23=25 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04k_c4_40_g25.log 2>&1"
for f in c4_50 c4_g40 c4_40 c4_g33 c4_50b c4_g40b c4_40b c4_40_g25; do echo -n "$f "; tail -n1 gpurun_out/r04k_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
