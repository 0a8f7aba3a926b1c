#!/bin/bash
# Round-2 GPU pass: whole GPU test suite (no -x: report every failure), then the bench in bf16
# and fp32. Each GPU step has its own time limit; a fault / abort / timeout ends the script.
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread ${1:+-k "$1"} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_bf16.json 2> gpurun_out/bench_bf16.err || exit $?
cat gpurun_out/bench_bf16.json
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --dtype fp32 > gpurun_out/bench_fp32.json 2> gpurun_out/bench_fp32.err || exit $?
cat gpurun_out/bench_fp32.json
exit $rc
