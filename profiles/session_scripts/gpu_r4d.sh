#!/bin/bash
# Round 4, session d: nx = 2 combine with every partner field fetched up front and the whole
# level at full EXEC (one select per value instead of masked regions): interleaved A/B against
# the committed build on c2 and the B = 1 pendulum probe, then the KKT / golden / IPM tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4d}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
B="--steps 100 --warmup 10 --no-cpu --no-ipm --problem pendulum --horizon 100 --batch 1024"
for i in 1 2 3; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_c2_$i.txt python bench.py $B
  run 0 200 new_c2_$i.txt python bench.py $B
done
NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_c2_ipm.txt python bench.py --steps 10 --warmup 2 --no-cpu --problem pendulum --horizon 100 --batch 1024
run 0 200 new_c2_ipm.txt python bench.py --steps 10 --warmup 2 --no-cpu --problem pendulum --horizon 100 --batch 1024
NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_wide.txt python tools/wide_probe.py pendulum:100 pendulum:400
run 0 200 new_wide.txt python tools/wide_probe.py pendulum:100 pendulum:400
run 1 900 pytest.txt python -u -m pytest tests/test_kkt_gpu.py tests/test_golden_gpu.py tests/test_ipm_gpu.py tests/test_api_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
