set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_v4
L=complexity-tokenizer_amd/complexity_tokenizer/libctok.so
bash tools/ab.sh $L $L,CTOK_DBG_MODE=20 > gpurun_out/r03_v4/ab_c4_noglobal.txt 2>&1
cat gpurun_out/r03_v4/ab_c4_noglobal.txt
CTOK_DBG_MODE=23 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r03_v4/dbg23.json 2> gpurun_out/r03_v4/dbg23.log
grep "ctok dbg" gpurun_out/r03_v4/dbg23.log | tail -3
