#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "gpurun_out/$log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run 200 ablate64.log python tools/kkt_ablate.py cartpole 200 4096 64
run 200 ablate32.log python tools/kkt_ablate.py cartpole 200 4096 32
run 120 counters_list.log rocprofv3 -L
run 300 prof_mem.log rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d "$R/gpurun_out/prof/mem" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu
run 300 prof_l2.log rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$R/gpurun_out/prof/l2" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu
