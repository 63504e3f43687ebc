#!/bin/bash
# KKT-scan parity tests, phase ablation (graph-replayed) and a kernel-trace profile of the c2 bench.
# Usage (repo root, via gpurun): gpurun --timeout 900 -- bash tools/gpu_ablate.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/abl; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 pytest_kkt.log python -u -m pytest tests/test_kkt_gpu.py -x -q --timeout 120 --timeout-method thread
run 200 c2.log python tools/kkt_ablate.py pendulum 100 1024 64
run 200 c2_l32.log python tools/kkt_ablate.py pendulum 100 1024 32
run 200 c3.log python tools/kkt_ablate.py cartpole 200 4096 32
run 200 bench_c2.log python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --cpu-seconds 5
run 200 prof_c2.log rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run -- python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --no-cpu --no-ipm
