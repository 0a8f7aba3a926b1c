#!/bin/bash
# igemm3 tile order (DCGAN_IGEMM_NMAJOR: a = per-launch footprint heuristic, 0 = M slowest, 1 = N
# slowest): GPU suite first, then the headline A/B and the 256x256 fp16 config
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_nmajor.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests_nmajor.log; [ $rc -eq 0 ] || exit $rc
./scripts/gpu_ab_vals.sh DCGAN_IGEMM_NMAJOR "a 0 1" || exit 1
for i in 1 2; do for v in a 0; do
  r=$(DCGAN_IGEMM_NMAJOR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --output_size 256 --batch_size 512 --dtype fp16 2>/dev/null) || exit 1
  echo "[256 fp16 NMAJOR=$v] $(echo "$r" | python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"])')"
done; done | tee gpurun_out/ab_nmajor_256.txt
