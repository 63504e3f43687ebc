#!/bin/bash
# A/B of the nx=8 group solve: library built with DPP group broadcasts (default) vs the
# ds_bpermute build (libnoc_hip_old.so); GPU tests on the default first.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/ab_c4; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
C4="--problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --no-cpu --no-ipm"
run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old1.log python bench.py $C4
run 200 new1.log python bench.py $C4
NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old2.log python bench.py $C4
run 200 new2.log python bench.py $C4
run 200 c4_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/c4_trace" -o run -- python "$R/bench.py" $C4
