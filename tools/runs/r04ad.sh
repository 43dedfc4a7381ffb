# stem chunk count: C5 pairs 4 (default) vs 2, C2 4 vs 2
b() { echo "200 env $1 python bench.py --model $3 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04ad_$2.log 2>&1"; }
tools/gpu_steps.sh "$(b RN_X=0 c5d1 resnet50_int8)" "$(b RN_STEM_CHUNKS=2 c5h1 resnet50_int8)" "$(b RN_X=0 c5d2 resnet50_int8)" "$(b RN_STEM_CHUNKS=2 c5h2 resnet50_int8)" \
  "$(b RN_X=0 c2d resnet50)" "$(b RN_STEM_CHUNKS=2 c2h resnet50)"
for f in c5d1 c5h1 c5d2 c5h2 c2d c2h; do echo -n "$f "; tail -n1 gpurun_out/r04ad_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
