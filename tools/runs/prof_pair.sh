# rocprofv3 kernel traces of the bench step: two streams (default) and one stream (per-kernel times alone)
tag=${1:-x2}
tools/gpu_steps.sh \
 "240 bash tools/prof_bench.sh ${tag} --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_prof.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh ${tag}1s --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}1s_prof.log 2>&1"
