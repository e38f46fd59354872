set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03_v7
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 400 python -u tools/bench_matrix.py --configs c3,c3tt --kernel-only --out $OUT/matrix_c3.json > $OUT/matrix.log 2>&1 || { tail -30 $OUT/matrix.log; exit 1; }
grep "\[matrix\]" $OUT/matrix.log
timeout -k 10 200 python -u tools/load_time.py $OUT/load_time.json > $OUT/load_time.log 2>&1 || { tail -20 $OUT/load_time.log; exit 1; }
cat $OUT/load_time.log
