#!/bin/bash
# PMC counters over whole training steps (eager launches: every dispatch counted), two passes
# (kernel-trace + counters only), summarised by scripts/pmc_summary2.py. BENCH_ARGS: extra bench.py
# arguments (e.g. "--output_size 256 --batch_size 512 --dtype fp16"); OUT: summary file name.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmcs1 gpurun_out/pmcs2
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcs1 -o p \
  --pmc SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  -- python3 bench.py --graph 0 --steps 7 --warmup 2 $BENCH_ARGS > gpurun_out/pmcs1.log 2>&1 || { tail -30 gpurun_out/pmcs1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcs2 -o p \
  --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY FETCH_SIZE \
  -- python3 bench.py --graph 0 --steps 7 --warmup 2 $BENCH_ARGS > gpurun_out/pmcs2.log 2>&1 || { tail -30 gpurun_out/pmcs2.log; exit 1; }
python3 scripts/pmc_summary2.py $(find gpurun_out/pmcs1 -name '*counter_collection.csv') $(find gpurun_out/pmcs2 -name '*counter_collection.csv') \
  > gpurun_out/${OUT:-step_pmc.txt} && head -40 gpurun_out/${OUT:-step_pmc.txt}
