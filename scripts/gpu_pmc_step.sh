#!/bin/bash
# PMC counters over whole training steps (eager launches, so every dispatch is counted):
# pass 1 = MFMA instruction count / LDS bank conflicts, pass 2 = HBM fetch bytes. Kernel-trace + counters only.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcs1 -o p \
  --pmc SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  -- python3 bench.py --graph 0 --steps 5 --warmup 2 > gpurun_out/pmcs1.log 2>&1 || { tail -30 gpurun_out/pmcs1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcs2 -o p \
  --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  -- python3 bench.py --graph 0 --steps 5 --warmup 2 > gpurun_out/pmcs2.log 2>&1 || { tail -30 gpurun_out/pmcs2.log; exit 1; }
find gpurun_out/pmcs1 gpurun_out/pmcs2 -name '*.csv' | head -20
