#!/bin/bash
# PMC counters for one conv-GEMM shape (kernel-trace + counters only; no other trace domains)
# usage: gpu_pmc.sh SHAPE CFGS [TAG]   (DCGAN_IGEMM_ABLATE in the environment is honoured)
SHAPE=${1:-D1.fwd}; CFGS=${2:-210:1}; TAG=${3:-pmc}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}1 -o p \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -- python3 benchmarks/kprobe.py --shape "$SHAPE" --cfgs "$CFGS" --reps 3 > gpurun_out/${TAG}1.log 2>&1 || { tail -30 gpurun_out/${TAG}1.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}2 -o p \
  --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
  -- python3 benchmarks/kprobe.py --shape "$SHAPE" --cfgs "$CFGS" --reps 3 > gpurun_out/${TAG}2.log 2>&1 || { tail -30 gpurun_out/${TAG}2.log; exit 1; }
python3 scripts/pmc_kernel.py $(find gpurun_out/${TAG}1 gpurun_out/${TAG}2 -name '*counter_collection.csv')
