#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r16; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "$O/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_all.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 300 sweep_c4.log python tools/kkt_sweep.py --configs c4 --lanes 1 --layouts tiled,natural --rounds 3 --reps 3
run 300 bench_c4.log python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --no-cpu
run 200 ipm_lin8.log python tools/ipm_bench.py linear8 512 2048 multi
