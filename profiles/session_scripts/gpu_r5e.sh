#!/bin/bash
# Round 5, session e: where the one-wave-per-SIMD scan's time goes -- SQ wait / issue counters and
# the instruction cache (SQC) for the 1024 shard, c2 and c3 (one --pmc pass per block).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5e}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 60 counters_list.log timeout -s KILL 50 rocprofv3 -L
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
SQ2="SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES"
SQC="SQC_ICACHE_REQ SQC_ICACHE_MISSES"
for c in s1024 c2 c3; do
  case $c in
    c3) A="--steps 20 --warmup 2" ;;
    c2) A="--problem pendulum --horizon 100 --batch 1024 --steps 50 --warmup 5" ;;
    s1024) A="--batch 1024 --steps 50 --warmup 5" ;;
  esac
  A="$A --no-cpu --no-ipm"
  run 120 ${c}_sq.log timeout -s KILL 110 rocprofv3 --pmc $SQ --output-format csv -d "$R/$O/${c}_sq" -o run -- python "$R/bench.py" $A
  python tools/pmc_mean.py $O/${c}_sq/run_counter_collection.csv > $O/${c}_sq_mean.json
  for k in $SQ2; do grep -q "$k" $O/counters_list.log || SQ2="${SQ2/$k/}"; done
  run 120 ${c}_sq2.log timeout -s KILL 110 rocprofv3 --pmc $SQ2 --output-format csv -d "$R/$O/${c}_sq2" -o run -- python "$R/bench.py" $A
  python tools/pmc_mean.py $O/${c}_sq2/run_counter_collection.csv > $O/${c}_sq2_mean.json
  if grep -q SQC_ICACHE_MISSES $O/counters_list.log; then
    run 120 ${c}_sqc.log timeout -s KILL 110 rocprofv3 --pmc $SQC --output-format csv -d "$R/$O/${c}_sqc" -o run -- python "$R/bench.py" $A
    python tools/pmc_mean.py $O/${c}_sqc/run_counter_collection.csv > $O/${c}_sqc_mean.json
  fi
done
