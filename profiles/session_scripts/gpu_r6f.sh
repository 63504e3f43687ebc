#!/bin/bash
# Round 6, session f: phases 1 / 3 of the persistent solver's KKT scan with one stage of compact
# blocks in flight (PF, the default build) against the same build without (libnoc_hip_nopf.so,
# -DNOC_PERSIST_PF=0), interleaved: c3, 512 and 1 cart-poles; the bit-identity tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6f; mkdir -p $O
export TMPDIR=/tmp
L=$R/ip-parallel-optimal-control_amd/noc/_lib
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }

for rnd in 1 2 3; do
  NOC_ALLOW_STALE_LIB=1 NOC_HIP_LIB=$L/libnoc_hip_nopf.so run 120 nopf_c3_$rnd.log python tools/ipm_bench.py cartpole 200 4096 persistent
  run 120 pf_c3_$rnd.log python tools/ipm_bench.py cartpole 200 4096 persistent
  NOC_ALLOW_STALE_LIB=1 NOC_HIP_LIB=$L/libnoc_hip_nopf.so NOC_PERSIST_WIDE=0 run 120 nopf_512_$rnd.log python tools/ipm_bench.py cartpole 200 512 persistent
  NOC_PERSIST_WIDE=0 run 120 pf_512_$rnd.log python tools/ipm_bench.py cartpole 200 512 persistent
done
NOC_ALLOW_STALE_LIB=1 NOC_HIP_LIB=$L/libnoc_hip_nopf.so NOC_PERSIST_WIDE=0 run 120 nopf_1.log python tools/ipm_bench.py cartpole 200 1 persistent
NOC_PERSIST_WIDE=0 run 120 pf_1.log python tools/ipm_bench.py cartpole 200 1 persistent
