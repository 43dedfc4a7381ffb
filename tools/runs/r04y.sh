# C4: weight-gradient split percent 45 (default) vs 40 / 35, pairs
b() { echo "200 env $1 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04y_$2.log 2>&1"; }
tools/gpu_steps.sh "$(b RN_X=0 d1)" "$(b RN_TUNE=21=40 s40a)" "$(b RN_TUNE=21=35 s35a)" "$(b RN_X=0 d2)" "$(b RN_TUNE=21=40 s40b)" "$(b RN_TUNE=21=35 s35b)"
for f in d1 s40a s35a d2 s40b s35b; do echo -n "$f "; tail -n1 gpurun_out/r04y_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
