#!/bin/bash
# One GPU-box session (run through gpurun from the repo root): GPU parity tests, the default
# bench line (with the CPU baseline), a rocprofv3 kernel-trace summary of the same bench, and the
# two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic per launch.  Every GPU step has its own
# time limit and the steps are chained so that the first failure ends the session.
#   usage: bash tools/gpu_check.sh TAG [tests|notests|profonly] [pmc|nopmc]
set -e
TAG=${1:-run}
TESTS=${2:-tests}
PMC=${3:-pmc}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$TESTS" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
if [ "$TESTS" != profonly ]; then
  timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -20 "$OUT/bench.log"; exit 1; }
  cat "$OUT/bench.json"
fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/bench.py" --steps 10 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.log" \
  || { tail -20 "$OUT/prof_bench.log"; exit 1; }
cat "$OUT/prof_bench.json"
if [ "$PMC" = pmc ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --corpus-workers 1 > "$OUT/pmc_fetch.log" 2>&1 \
    || { tail -20 "$OUT/pmc_fetch.log"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --corpus-workers 1 > "$OUT/pmc_write.log" 2>&1 \
    || { tail -20 "$OUT/pmc_write.log"; exit 1; }
  python3 "$ROOT/tools/pmc_traffic.py" "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json" c4/10000000
fi
echo "gpu_check $TAG done"
