#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; cd gpurun_out
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_VALU SQ_WAIT_ANY -d pmc_c3a -o run -- python -m benchmarks.bench_narrow > pmc_c3.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d pmc_c3b -o run -- python -m benchmarks.bench_narrow >> pmc_c3.log 2>&1 || exit 1
