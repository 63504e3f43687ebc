#!/bin/bash
# Round 6, session h: LDS bank conflicts of the persistent solver (the trajectory's states /
# controls and the KKT slots are lane-strided in LDS): SQ_LDS_BANK_CONFLICT against
# SQ_LDS_IDX_ACTIVE, at 512 cart-poles (one wave per SIMD) and c3.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6h; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU"
NOC_PERSIST_WIDE=0 run 150 lds512.log timeout -s KILL 140 rocprofv3 --pmc $C --output-format csv -d "$R/$O/lds512" -o run -- python $R/tools/ipm_bench.py cartpole 200 512 persistent
python tools/pmc_mean.py $O/lds512/run_counter_collection.csv ipm_solve_kernel > $O/lds512_mean.json
run 150 ldsc3.log timeout -s KILL 140 rocprofv3 --pmc $C --output-format csv -d "$R/$O/ldsc3" -o run -- python $R/tools/ipm_bench.py cartpole 200 4096 persistent
python tools/pmc_mean.py $O/ldsc3/run_counter_collection.csv ipm_solve_kernel > $O/ldsc3_mean.json
cat $O/*_mean.json
