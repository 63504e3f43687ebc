#!/bin/bash
# One GPU session: parity tests, smoke, the three bench lines (c3 default, c2, c4) and the
# end-to-end solve timings.  Usage (from the repo root, via gpurun):
#   gpurun --timeout 1200 -- bash tools/gpu_check.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/check; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 200 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench_c3.log python bench.py
run 300 bench_c2.log python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --cpu-seconds 5
run 300 bench_c4.log python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --cpu-seconds 10 --cpu-sample 256
run 300 runtime_pend.log python tools/runtime_sweep.py --problem pendulum --out $O/runtime
run 300 runtime_cart.log python tools/runtime_sweep.py --problem cartpole --out $O/runtime
