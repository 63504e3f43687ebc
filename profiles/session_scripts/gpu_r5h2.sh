#!/bin/bash
# Heavy-first split of the c3 persistent solve (NOC_PERSIST_HEAVY): interleaved A/B of the
# heavy count, u hash for bit-identity, plus the per-trajectory computed solves / launch order.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5h2}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
for r in 1 2; do
  for h in ${HEAVY_LIST:-0 32 64 128 256}; do
    NOC_PERSIST_HEAVY=$h run 120 ipm_h${h}_$r.json python tools/ipm_bench.py cartpole 200 4096 persistent
  done
done
