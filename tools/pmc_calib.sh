#!/bin/bash
# FETCH_SIZE calibration (profiling helper): two PMC passes over tools/fetch_calib, then the
# tallied bytes per known byte / access of every shape.   usage: bash tools/pmc_calib.sh OUTDIR
out=$1; ROOT=$(pwd)
mkdir -p "$out"
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$out/calib_fetch" -o run -- \
    "$ROOT/tools/fetch_calib" > "$ROOT/$out/calib_fetch.log" 2>&1 ) || { tail -5 "$out/calib_fetch.log"; exit 1; }
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum \
    --output-format csv -d "$ROOT/$out/calib_req" -o run -- "$ROOT/tools/fetch_calib" > "$ROOT/$out/calib_req.log" 2>&1 ) \
  || { tail -5 "$out/calib_req.log"; exit 1; }
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/$out/calib_write" -o run -- \
    "$ROOT/tools/fetch_calib" > "$ROOT/$out/calib_write.log" 2>&1 ) || { tail -5 "$out/calib_write.log"; exit 1; }
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum \
    --output-format csv -d "$ROOT/$out/calib_wreq" -o run -- "$ROOT/tools/fetch_calib" > "$ROOT/$out/calib_wreq.log" 2>&1 ) \
  || { tail -5 "$out/calib_wreq.log"; exit 1; }
python3 "$ROOT/tools/pmc_calib_report.py" "$out" | tee "$out/fetch_calibration.txt"
