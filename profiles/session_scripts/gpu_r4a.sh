#!/bin/bash
# Round 4, session a: every GPU test (the device check_traj_feasibility, the max_steps cap, the
# one-allocation workspace, the wave-scope fence of the scan's copy-out), smoke, the c3 bench line,
# the strong-scaling rehearsals on one GPU (world 2 / 4 over gloo: the ipm_solve totals must equal
# the 1-rank line now that every rank shards one global batch), the B = 1 probe and runtime sweeps.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4a}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 0 200 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
run 0 300 bench_c3.txt python bench.py
run 0 300 rehearsal_w2.txt env NOC_BENCH_REHEARSAL=1 python bench.py --gpus 2 --steps 10 --no-cpu
run 0 300 rehearsal_w4.txt env NOC_BENCH_REHEARSAL=1 python bench.py --gpus 4 --steps 10 --no-cpu
run 0 300 wide.txt python tools/wide_probe.py cartpole:100 cartpole:200 pendulum:100 pendulum:400
run 0 400 runtime_pendulum.txt python tools/runtime_sweep.py --problem pendulum --out $O/runtime --runs 5
run 0 400 runtime_cartpole.txt python tools/runtime_sweep.py --problem cartpole --out $O/runtime --runs 5
