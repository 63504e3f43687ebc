#!/bin/bash
# Where the persistent solver's time goes at c3: SQ issue / wait counters and the calibrated
# FETCH_SIZE / WRITE_SIZE traffic of ipm_solve_kernel (one --pmc pass per block), plus its trace.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5q1}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
SQ2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_MISC"
CMD="python $R/tools/ipm_bench.py cartpole 200 4096 persistent"
run 150 trace.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- $CMD
run 150 sq.log timeout -s KILL 140 rocprofv3 --pmc $SQ --output-format csv -d "$R/$O/sq" -o run -- $CMD
python tools/pmc_mean.py $O/sq/run_counter_collection.csv ipm_solve_kernel > $O/sq_mean.json
run 150 sq2.log timeout -s KILL 140 rocprofv3 --pmc $SQ2 --output-format csv -d "$R/$O/sq2" -o run -- $CMD
python tools/pmc_mean.py $O/sq2/run_counter_collection.csv ipm_solve_kernel > $O/sq2_mean.json
run 150 fetch.log timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/fetch" -o run -- $CMD
python tools/pmc_mean.py $O/fetch/run_counter_collection.csv ipm_solve_kernel > $O/fetch_mean.json
run 150 write.log timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/write" -o run -- $CMD
python tools/pmc_mean.py $O/write/run_counter_collection.csv ipm_solve_kernel > $O/write_mean.json
cat $O/*_mean.json
