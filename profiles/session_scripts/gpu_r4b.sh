#!/bin/bash
# Round 4, session b: (1) the new / fixed GPU tests (engine reuse, the max_steps cap);
# (2) interleaved A/B of the scan's copy-out ordering: libnoc_hip_old.so (workgroup barrier) vs
# the default build (wave-scope fence for one-wave segments) on c3, c2 and the 512 shard;
# (3) the B = 1 probe and the reference's runtime sweeps with the reused engines.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4b}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 600 pytest_new.txt python -u -m pytest tests/test_ipm_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf -k "cached_engine or max_steps or cap"
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2; do
  for c in "c3:" "c2:--problem pendulum --horizon 100 --batch 1024" "s512:--global-batch 512"; do
    n=${c%%:*}; a=${c#*:}
    NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_${n}_$i.txt python bench.py $B $a
    run 0 200 new_${n}_$i.txt python bench.py $B $a
  done
done
run 0 300 wide.txt python tools/wide_probe.py cartpole:100 cartpole:200 pendulum:100 pendulum:400
run 0 400 runtime_pendulum.txt python tools/runtime_sweep.py --problem pendulum --out $O/runtime --runs 5
run 0 400 runtime_cartpole.txt python tools/runtime_sweep.py --problem cartpole --out $O/runtime --runs 5
