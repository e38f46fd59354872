set -e
mkdir -p gpurun_out/t1
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1/gpu_tests.log 2>&1 || { tail -40 gpurun_out/t1/gpu_tests.log; exit 1; }
tail -3 gpurun_out/t1/gpu_tests.log
L=complexity-tokenizer_amd/complexity_tokenizer/libctok.so
bash tools/ab.sh $L $L,CTOK_FORCE_WIDE_SLOTS=1 --config c2
