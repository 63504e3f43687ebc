#!/bin/bash
# Round 5: phase 3's last reads non-temporal (NOC_KKT_NT3=1, "nt") vs the default cache policy
# (NOC_KKT_NT3=0, "def"), same build, interleaved bench lines (graph-replayed steps).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r5w; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
declare -A ARGS=([c3]="" [c5]="--batch 8192" [n300]="--horizon 300" [b16k]="--batch 16384" [s2048]="--global-batch 2048" [s1024]="--global-batch 1024" [s512]="--global-batch 512" [n100]="--horizon 100")
for i in 1 2 3; do
  for c in c3 c5 n300 b16k s2048 s1024 s512 n100; do
    NOC_KKT_NT3=0 run 200 def_${c}_$i.log python bench.py $B ${ARGS[$c]}
    NOC_KKT_NT3=1 run 200 nt_${c}_$i.log python bench.py $B ${ARGS[$c]}
  done
done
