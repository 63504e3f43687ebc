#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (tools/pmc_calib.hip, known byte counts per access width)
# and a refreshed per-launch counter pass of the c3 bench kernel, one counter group per run.
R="${GRAFT_REPO_ROOT:-/root/repo}"
O=$R/gpurun_out/pmc_calib; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() { local log=$1; shift; timeout -s KILL 120 "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run calib_fetch.log rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- $R/tools/pmc_calib
run calib_write.log rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- $R/tools/pmc_calib
run calib_req.log rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/calib_req -o run --output-format csv -- $R/tools/pmc_calib
run c3_fetch.log rocprofv3 --pmc FETCH_SIZE -d $O/c3_fetch -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --no-ipm
run c3_write.log rocprofv3 --pmc WRITE_SIZE -d $O/c3_write -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --no-ipm
run c3_req.log rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/c3_req -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --no-ipm
