#!/bin/bash
# Round-2 evidence: (1) tile sweep incl. igemm v1 (LDS-DMA variants) vs igemm3 4/8-wave tiles,
# (2) kernel-trace profile of the graph-launched bench step, (3) per-kernel PMC over eager steps.
mkdir -p gpurun_out
timeout -k 10 700 python -u benchmarks/bench_kernels.py --batch 128 --reps 10 --top 8 --v1 --cfgs 1,2 \
  --out gpurun_out/tuned_v1v3.json > gpurun_out/tune_v1v3.log 2>&1 || { tail -20 gpurun_out/tune_v1v3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/tune_v1v3.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
rm -rf gpurun_out/prof_r2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2 -o run -- python3 bench.py --steps 20 --warmup 5 \
  > gpurun_out/prof_r2.log 2>&1 || { tail -20 gpurun_out/prof_r2.log; exit 1; }
tail -2 gpurun_out/prof_r2.log
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcr2a -o p \
  --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  -- python3 bench.py --graph 0 --steps 5 --warmup 2 > gpurun_out/pmcr2a.log 2>&1 || { tail -20 gpurun_out/pmcr2a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcr2b -o p \
  --pmc FETCH_SIZE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -- python3 bench.py --graph 0 --steps 5 --warmup 2 > gpurun_out/pmcr2b.log 2>&1 || { tail -20 gpurun_out/pmcr2b.log; exit 1; }
find gpurun_out/prof_r2 gpurun_out/pmcr2a gpurun_out/pmcr2b -type f | head -20
