#!/bin/bash
# Round-3 closing measurements on one MI355X: GPU tests, the bench line (C4 and C2), a rocprofv3
# kernel trace of the bench command, the FETCH_SIZE / WRITE_SIZE passes for the traffic field,
# and the config matrix.  Every GPU step has its own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
OUT=$(pwd)/gpurun_out/${TAG:-r03_final}
mkdir -p "$OUT"
ROOT=$(pwd)
STEP=${1:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -20 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.json"
  timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.log" || { tail -20 "$OUT/bench_c2.log"; exit 1; }
  tail -1 "$OUT/bench_c2.json"
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --corpus-workers 1 > "$OUT/pmc_fetch.log" 2>&1 || { tail -20 "$OUT/pmc_fetch.log"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --corpus-workers 1 > "$OUT/pmc_write.log" 2>&1 || { tail -20 "$OUT/pmc_write.log"; exit 1; }
  cd "$ROOT"
  python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json" c4/10000000 > "$OUT/pmc_traffic.log"
  cat "$OUT/pmc_traffic.log"
fi
if [ "$STEP" = all ] || [ "$STEP" = matrix ]; then
  timeout -k 10 900 python -u tools/bench_matrix.py --configs c1,c2,c3,c3tt,c5,c5nfc --out "$OUT/matrix.json" > "$OUT/matrix.log" 2>&1 || { tail -30 "$OUT/matrix.log"; exit 1; }
  grep "\[matrix\]" "$OUT/matrix.log" | grep done
fi
echo "r03_final $STEP done"
