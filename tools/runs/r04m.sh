# main-stream priority and the split percent near its optimum (C2 pairs)
b() { echo "200 env $1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04m_$2.log 2>&1"; }
tools/gpu_steps.sh \
 "$(b RN_X=0 d1)" "$(b RN_MAIN_PRIORITY=0 noprio)" "$(b RN_TUNE=21=45 s45)" "$(b RN_TUNE=21=55 s55)" \
 "$(b RN_X=0 d2)" "$(b RN_MAIN_PRIORITY=0 noprio2)" "$(b RN_TUNE=21=45 s45b)" "$(b RN_TUNE=21=55 s55b)"
for f in d1 noprio s45 s55 d2 noprio2 s45b s55b; do echo -n "$f "; tail -n1 gpurun_out/r04m_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
