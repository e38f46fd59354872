set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_v5
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r03_v5/warm.json 2> gpurun_out/r03_v5/warm.log
bash tools/pmc_sq.sh v5a c4 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
bash tools/pmc_sq.sh v5b c4 "SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
