#!/bin/bash
# Round 6 final, part b: same-build kernel traces + calibrated FETCH_SIZE / WRITE_SIZE passes of
# every bench configuration (c3, c2, c4, c5 and the strong-scaling shards), written to
# $O/prof/pmc_traffic.json stamped with the KKT source hash, then the shard and c5 bench lines on
# those stamps.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r6final_b}; mkdir -p $O
export TMPDIR=/tmp
OUT=${OUT:-r6final_b}/prof bash profiles/session_scripts/gpu_final_r3.sh || exit 1
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
P="--pmc-json $O/prof/pmc_traffic.json --no-cpu"
run 300 bench_c5.txt python bench.py --batch 8192 --steps 20 --warmup 2 $P
run 300 bench_s2048.txt python bench.py --batch 2048 $P
run 300 bench_s1024.txt python bench.py --batch 1024 $P
run 300 bench_s512.txt python bench.py --batch 512 $P
run 300 bench_c4.txt python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 $P
