#!/bin/bash
# End-of-session validation: all GPU tests, smoke, c3 kernel trace + HBM PMC passes, and the
# three bench lines (c3 is the driver's default command).  gpurun --timeout 1200 -- bash tools/gpu_final.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/final3; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
C3="--steps 20 --warmup 2 --no-cpu --no-ipm"
run 700 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run 200 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 200 c2_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/c2_trace" -o run -- python "$R/bench.py" --problem pendulum --horizon 100 --batch 1024 --steps 50 --warmup 5 --no-cpu --no-ipm
run 200 c3_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/c3_trace" -o run -- python "$R/bench.py" $C3
run 120 c3_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/c3_fetch" -o run -- python "$R/bench.py" $C3
run 120 c3_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/c3_write" -o run -- python "$R/bench.py" $C3
cp profiles/pmc_traffic.json $O/pmc_traffic.json
python tools/pmc_traffic.py $O/c3_fetch/run_counter_collection.csv $O/c3_write/run_counter_collection.csv cartpole_N200_B4096 $O/pmc_traffic.json kkt_scan
run 300 bench_c3.log python bench.py
run 300 bench_c2.log python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --cpu-seconds 5
run 300 bench_c4.log python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --cpu-seconds 10 --cpu-sample 256
