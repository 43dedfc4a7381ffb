# round 3: rocprofv3 kernel traces of C2 / C4 / C5 (two streams, default knobs) + C5 / C4 bench lines
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for m in resnet50 resnext50 resnet50_int8; do
  rm -rf gpurun_out/prof_r03g_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03g_$m -o run --output-format csv -- python3 bench.py --model $m --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03g_prof_$m.json 2> gpurun_out/r03g_prof_$m.err || { echo "prof $m failed"; tail -5 gpurun_out/r03g_prof_$m.err; exit 1; }
  f=$(find gpurun_out/prof_r03g_$m -name "*kernel_trace.csv" | head -1)
  python3 tools/step_breakdown.py $f > gpurun_out/r03g_breakdown_$m.txt || exit 1
  head -25 gpurun_out/r03g_breakdown_$m.txt
done
for m in resnext50 resnet50_int8; do
  timeout -k 10 300 python bench.py --model $m --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03g_bench_$m.json 2> gpurun_out/r03g_bench_$m.err || exit 1
  tail -c 400 gpurun_out/r03g_bench_$m.json
done
