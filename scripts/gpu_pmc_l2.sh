#!/bin/bash
# L2 (TCC) hit rate and request counts per kernel over eager training steps (kernel-trace +
# counters only), then the counter list of this GPU for reference.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmcl2
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc_list_avail.txt 2>&1 || true
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcl2 -o p \
  --pmc TCC_HIT_sum TCC_MISS_sum \
  -- python3 bench.py --graph 0 --steps 7 --warmup 2 $BENCH_ARGS > gpurun_out/pmcl2.log 2>&1 || { tail -30 gpurun_out/pmcl2.log; exit 1; }
python3 scripts/pmc_generic.py $(find gpurun_out/pmcl2 -name '*counter_collection.csv') > gpurun_out/step_pmc_l2.txt && head -40 gpurun_out/step_pmc_l2.txt
