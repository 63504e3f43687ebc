#!/bin/bash
# Profile refresh after the cached-chunk scan (c2) and the 8-waves/CU group solve (c4): GPU tests,
# kernel traces, HBM PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs) for c2 and c4, and
# the three bench lines.  Usage (repo root, via gpurun): gpurun --timeout 1200 -- bash tools/gpu_profile.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/profile; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
C2="--problem pendulum --horizon 100 --batch 1024 --steps 50 --warmup 5 --no-cpu --no-ipm"
C3="--steps 20 --warmup 2 --no-cpu --no-ipm"
C4="--problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 5 --warmup 1 --no-cpu --no-ipm"
run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 200 c2_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/c2_trace" -o run -- python "$R/bench.py" $C2
run 200 c3_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/c3_trace" -o run -- python "$R/bench.py" $C3
run 300 c4_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/c4_trace" -o run -- python "$R/bench.py" $C4
run 120 c2_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/c2_fetch" -o run -- python "$R/bench.py" $C2
run 120 c2_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/c2_write" -o run -- python "$R/bench.py" $C2
run 200 c4_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/c4_fetch" -o run -- python "$R/bench.py" $C4
run 200 c4_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/c4_write" -o run -- python "$R/bench.py" $C4
cp profiles/pmc_traffic.json $O/pmc_traffic.json
python tools/pmc_traffic.py $O/c2_fetch/run_counter_collection.csv $O/c2_write/run_counter_collection.csv pendulum_N100_B1024 $O/pmc_traffic.json kkt_scan
python tools/pmc_traffic.py $O/c4_fetch/run_counter_collection.csv $O/c4_write/run_counter_collection.csv linear8_N512_B16384 $O/pmc_traffic.json kkt_group8
# only gpurun_out/ comes back from the box: merge $O/pmc_traffic.json into profiles/pmc_traffic.json by hand
run 300 bench_c3.log python bench.py
run 300 bench_c2.log python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --cpu-seconds 5
run 300 bench_c4.log python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --cpu-seconds 10 --cpu-sample 256
