#!/bin/bash
# Round 3 final validation of the committed tree: every GPU test, smoke(), the driver's default
# bench line (c3, with cpu_baseline and ipm_solve), the c2 / c4 bench lines, the strong-scaling
# rehearsal at world 2 (gloo, all ranks on cuda:0: timings meaningless) and the B = 1 runtime
# sweeps of the reference's timing harness.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-final_r3b}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 0 300 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
run 0 300 bench_c3.txt python bench.py
run 0 300 bench_c2.txt python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --cpu-seconds 5
run 0 300 bench_c4.txt python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --cpu-seconds 10 --cpu-sample 256
run 0 200 rehearsal_w2.txt env NOC_BENCH_REHEARSAL=1 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu
run 0 400 runtime_pendulum.txt python tools/runtime_sweep.py --problem pendulum --out $O/runtime --runs 5
run 0 400 runtime_cartpole.txt python tools/runtime_sweep.py --problem cartpole --out $O/runtime --runs 5
