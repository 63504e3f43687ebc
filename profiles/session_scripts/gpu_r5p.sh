#!/bin/bash
# Round 5, session p: instruction-cache counters of the 512-shard and 1024-shard kernels, round-4
# library vs the current one (same L = 128 kernel bytes, different code placement).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5p}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ]; then exit $rc; fi; }
SQC="SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_HITS"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU"
for c in s512 s1024; do
  case $c in s512) A="--global-batch 512" ;; s1024) A="--global-batch 1024" ;; esac
  A="$A --steps 50 --warmup 5 --no-cpu --no-ipm"
  for v in old new; do
    case $v in new) lib=libnoc_hip.so ;; old) lib=libnoc_hip_old.so ;; esac
    NOC_HIP_LIB=$L/$lib run 120 ${v}_${c}_sqc.log timeout -s KILL 110 rocprofv3 --pmc $SQC --output-format csv -d "$R/$O/${v}_${c}_sqc" -o run -- python "$R/bench.py" $A
    python tools/pmc_mean.py $O/${v}_${c}_sqc/run_counter_collection.csv > $O/${v}_${c}_sqc_mean.json
    NOC_HIP_LIB=$L/$lib run 120 ${v}_${c}_sq.log timeout -s KILL 110 rocprofv3 --pmc $SQ --output-format csv -d "$R/$O/${v}_${c}_sq" -o run -- python "$R/bench.py" $A
    python tools/pmc_mean.py $O/${v}_${c}_sq/run_counter_collection.csv > $O/${v}_${c}_sq_mean.json
  done
done
