#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r22; mkdir -p $O
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-900; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 bench_c5_pergpu.log python bench.py --batch 8192 --steps 50 --warmup 5 --no-cpu
run 300 bench_default.log python bench.py
