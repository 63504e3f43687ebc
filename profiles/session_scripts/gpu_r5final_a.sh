#!/bin/bash
# Round 5 final, part a (after part b's PMC traffic is in profiles/pmc_traffic.json): every GPU
# test, smoke, the bench under torch.distributed.run with one rank (RCCL on the hardware), the
# default bench line (c3, CPU baseline, ipm_solve) and the c2 / c4 / shard bench lines.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5final_a}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 200 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench_torchrun1.txt python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu
run 300 bench_c3.txt python bench.py
run 300 bench_c2.txt python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --cpu-seconds 5
run 300 bench_c4.txt python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --cpu-seconds 10 --cpu-sample 256
for c in 2048 1024 512; do
  run 200 bench_s$c.txt python bench.py --global-batch $c --steps 50 --warmup 5 --no-cpu --no-ipm
done
run 200 bench_c5.txt python bench.py --batch 8192 --steps 20 --warmup 3 --no-cpu --no-ipm
