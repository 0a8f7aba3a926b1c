#!/bin/bash
# per-kernel PMC of the current training step (two counter passes over eager steps) -> pmc_summary2.py
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmcA gpurun_out/pmcB
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcA -o p \
  --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  -- python3 bench.py --graph 0 --steps 5 --warmup 2 > gpurun_out/pmcA.log 2>&1 || { tail -20 gpurun_out/pmcA.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcB -o p \
  --pmc FETCH_SIZE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -- python3 bench.py --graph 0 --steps 5 --warmup 2 > gpurun_out/pmcB.log 2>&1 || { tail -20 gpurun_out/pmcB.log; exit 1; }
find gpurun_out/pmcA gpurun_out/pmcB -name "*counter_collection.csv"
