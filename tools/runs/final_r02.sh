# round-2 consolidated measurement: bench line (CPU baseline + PCIe leg), rocprofv3 two-stream and
# one-stream kernel traces of the bench step, PMC passes (HBM bytes, MFMA busy, LDS conflicts)
tag=${1:-r02f}
tools/gpu_steps.sh \
 "300 python bench.py > gpurun_out/${tag}_bench.log 2>&1" \
 "240 bash tools/prof_bench.sh ${tag} --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_prof.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh ${tag}1s --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}1s_prof.log 2>&1" \
 "900 bash tools/pmc_bench.sh ${tag} --steps 3 --warmup 1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_pmc.log 2>&1"
