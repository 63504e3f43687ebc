#!/bin/bash
# Profile refresh: c4 grouped group solve (trace, HBM PMC, SQ), c3 trace, and the bench lines.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/prof_r1c; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "$O/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
C3="--steps 20 --warmup 2 --no-cpu --no-ipm"
C4="--problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 5 --warmup 1 --no-cpu --no-ipm"
run 300 c3_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/c3_trace" -o run -- python "$R/bench.py" $C3
run 300 c4_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/c4_trace" -o run -- python "$R/bench.py" $C4
run 200 c4_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/c4_fetch" -o run -- python "$R/bench.py" $C4
run 200 c4_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/c4_write" -o run -- python "$R/bench.py" $C4
run 200 c4_sq.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d "$R/$O/c4_sq" -o run -- python "$R/bench.py" $C4
cp profiles/pmc_traffic.json $O/pmc_traffic.json
python tools/pmc_traffic.py $O/c4_fetch/run_counter_collection.csv $O/c4_write/run_counter_collection.csv linear8_N512_B16384 $O/pmc_traffic.json kkt_group8
cp $O/pmc_traffic.json profiles/pmc_traffic.json
run 300 bench_c3.log python bench.py --steps 50 --warmup 5 --cpu-seconds 10
run 300 bench_c4.log python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --cpu-seconds 10 --cpu-sample 256
run 300 bench_c2.log python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --cpu-seconds 5
