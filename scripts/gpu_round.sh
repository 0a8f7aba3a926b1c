#!/bin/bash
# Re-entry / milestone validation: GPU suite (every failure reported), smoke, bench bf16 + fp32,
# kernel-trace step profile. Each GPU step has its own limit; a fault/abort/timeout ends the script.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread ${1:+-k "$1"} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_bf16.json 2> gpurun_out/bench_bf16.err || exit $?
cat gpurun_out/bench_bf16.json
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --dtype fp32 > gpurun_out/bench_fp32.json 2> gpurun_out/bench_fp32.err || exit $?
cat gpurun_out/bench_fp32.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_round
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_round -o run -- python3 bench.py --steps 20 --warmup 5 \
  > gpurun_out/prof_round.log 2>&1 || { tail -20 gpurun_out/prof_round.log; exit 1; }
tail -1 gpurun_out/prof_round.log
exit $rc
