#!/bin/bash
# After a lane-policy change: GPU tests, then bench lines at the default lanes over horizons
# (cart-pole B=4096) and the c2 / c3 defaults.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/policy; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for n in 50 100 150 300 400; do
  run 200 n$n.log python bench.py --horizon $n --steps 30 --warmup 3 --no-cpu --no-ipm
done
run 200 pend_b4096.log python bench.py --problem pendulum --horizon 100 --batch 4096 --steps 30 --warmup 3 --no-cpu --no-ipm
run 200 pend_b16384.log python bench.py --problem pendulum --horizon 100 --batch 16384 --steps 30 --warmup 3 --no-cpu --no-ipm
run 300 bench_c3.log python bench.py
run 300 bench_c2.log python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --cpu-seconds 5
