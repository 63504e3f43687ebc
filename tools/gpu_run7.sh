#!/bin/bash
# Round-1 profile session: kernel trace + stats of the bench, PMC traffic passes, final bench line.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/prof7
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "gpurun_out/$log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run 300 p7_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof7/trace" -o run -- python "$R/bench.py" --steps 50 --warmup 5 --no-cpu
run 300 p7_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof7/fetch" -o run -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu
run 300 p7_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof7/write" -o run -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu
run 300 p7_sq.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD --output-format csv -d "$R/gpurun_out/prof7/sq" -o run -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu
run 300 p7_ta.log rocprofv3 --pmc TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$R/gpurun_out/prof7/ta" -o run -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu
python tools/pmc_traffic.py gpurun_out/prof7/fetch/run_counter_collection.csv gpurun_out/prof7/write/run_counter_collection.csv cartpole_N200_B4096 gpurun_out/prof7/pmc_traffic.json
cp gpurun_out/prof7/pmc_traffic.json profiles/pmc_traffic.json
run 300 p7_bench.log python bench.py --steps 50 --warmup 5 --cpu-seconds 10
