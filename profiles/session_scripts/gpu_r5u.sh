#!/bin/bash
# Round 5: phase 3's last reads of Q, R, M, r, q as non-temporal loads (ablation bit 7 in this
# build), graph-replayed, same build for both variants.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r5u; mkdir -p $O
export TMPDIR=/tmp
export ABLATE_VARIANTS='{"full": 0, "nt_q": 128}'
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 240 c3.log python tools/kkt_ablate.py cartpole 200 4096 32
run 240 c5.log python tools/kkt_ablate.py cartpole 200 8192 32
run 240 n300.log python tools/kkt_ablate.py cartpole 300 4096 32
run 240 c3b.log python tools/kkt_ablate.py cartpole 200 4096 32
run 240 b16k.log python tools/kkt_ablate.py cartpole 200 16384 32
