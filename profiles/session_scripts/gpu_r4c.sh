#!/bin/bash
# Round 4, session c: every GPU test (incl. the RCCL world-1 sharded solves and the retuned
# indefinite-Q test), smoke, the bench under torch.distributed.run with one rank (RCCL process
# group on the hardware), then same-build kernel traces + calibrated PMC traffic for every bench
# configuration (profiles/session_scripts/gpu_final_r3.sh) and the c3 / c2 / c4 bench lines.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4c}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 0 200 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
run 0 300 bench_torchrun1.txt python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu
OUT=${OUT:-r4c}/prof bash profiles/session_scripts/gpu_final_r3.sh || exit 1
cp $O/prof/pmc_traffic.json profiles/pmc_traffic.json
run 0 300 bench_c3.txt python bench.py
run 0 300 bench_c2.txt python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --cpu-seconds 5
run 0 300 bench_c4.txt python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --cpu-seconds 10 --cpu-sample 256
