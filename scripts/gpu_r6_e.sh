#!/bin/bash
# round 6: narrow-deconv staging/prefetch (kernel + engine tests, A/B vs ab_old), D-merge prototype
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_engine.py -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r6e.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests_r6e.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for a in "--steps 200 --warmup 20" "--steps 20 --warmup 5"; do
    r=$(timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1; echo "[new $a] ${r:70:40}"
    r=$(cd ab_old && timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1; echo "[old $a] ${r:70:40}"
  done
done | tee gpurun_out/ab_narrow_prefetch_r6.txt
{ timeout -k 10 300 python -u benchmarks/study/dmerge_proto.py --rounds 3 --steps 200 --warmup 20 --tiles heur || exit 1
  timeout -k 10 300 python -u benchmarks/study/dmerge_proto.py --rounds 3 --steps 200 --warmup 20 --tiles same2b || exit 1
} 2>&1 | tee gpurun_out/dmerge_proto_r6.txt
