#!/bin/bash
# GPU session 2: parity matrix, lanes sweep, rocprofv3 kernel trace + HBM counters.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -4 "gpurun_out/$log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run 600 kkt_tests.log python -m pytest tests/test_kkt_gpu.py -q
run 300 sweep.log python tools/kkt_sweep.py --configs c3,c2,c4
run 300 prof_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/trace" -o run -- python "$R/bench.py" --steps 20 --warmup 3 --no-cpu
run 300 prof_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof/fetch" -o run -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu
run 300 prof_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof/write" -o run -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu
run 300 prof_valu.log rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d "$R/gpurun_out/prof/valu" -o run -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu
find gpurun_out/prof -name "*.csv" | head -30
