# same-box kernel breakdowns of C5 with / without the quantizer max from the conv epilogue's extremes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 bash tools/prof_bench.sh r03s_mm --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03s_prof_mm.log 2>&1 || exit $?
timeout -k 10 240 env RN_QUANT_BN_MM=0 bash tools/prof_bench.sh r03s_pass --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03s_prof_pass.log 2>&1 || exit $?
timeout -k 10 240 env RN_MM_NOSIGN=1 bash tools/prof_bench.sh r03s_nosign --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03s_prof_nosign.log 2>&1 || exit $?
for t in mm pass nosign; do python3 tools/step_breakdown.py gpurun_out/prof_r03s_$t/run_kernel_trace.csv > gpurun_out/r03s_breakdown_$t.txt; done
grep "kernel sum\|, 0, 1, 0, 0, 0>\|bnq_absmax" gpurun_out/r03s_breakdown_*.txt
