#!/bin/bash
# c4 group-solve iteration: parity of the KKT paths, the c4 bench line, a kernel-trace profile.
# Usage (repo root, via gpurun): gpurun --timeout 900 -- bash tools/gpu_c4.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/c4; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-700; if [ $rc -ne 0 ]; then exit $rc; fi; }
C4="--problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2"
run 300 pytest_kkt.log python -u -m pytest tests/test_kkt_gpu.py tests/test_ipm_gpu.py -x -q --timeout 120 --timeout-method thread
run 200 bench_c4.log python bench.py $C4 --cpu-seconds 5 --cpu-sample 64
run 200 prof_c4.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python bench.py $C4 --no-cpu --no-ipm
