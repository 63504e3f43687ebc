#!/bin/bash
# Round 3, session e: why two-wave segments (lanes 128) are slower at 512 / 1024 trajectories:
# per-wave stamps at 128 and 64 lanes, kernel traces.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3e}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 0 120 stamps_s512_L128.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 512 128
run 0 120 stamps_s512_L64.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 512 64
run 0 120 stamps_s256_L128.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 256 128
run 0 200 trace_512.txt rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace512" -o run -- python "$R/bench.py" --batch 512 --lanes 128 --steps 20 --warmup 2 --no-cpu --no-ipm --no-graph
