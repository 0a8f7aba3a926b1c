#!/bin/bash
# round 5, call D: native RCCL communicator tests, then eager / graph x schedules with it
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_hip_ddp.py -x -v --timeout 300 --timeout-method thread \
  -k "native or rccl or force_ddp or copies" > gpurun_out/ddp_tests_d.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/ddp_tests_d.log | tail -20; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/sched_native_r5d.txt; : > $out
val() { python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); c=d["config"]; print(d["value"], d["ms_per_step"], c["graphs_per_step"], c["schedule"], c["collectives"])'; }
for i in 1 2 3; do
  for spec in "--graph 1" "--graph 0" "--force_ddp --graph 1" "--force_ddp --graph 0" \
              "DCGAN_DDP_SCHEDULE=ddp --force_ddp --graph 1" "DCGAN_DDP_SCHEDULE=ddp --force_ddp --graph 0" \
              "DCGAN_NATIVE_RCCL=0 DCGAN_DDP_SCHEDULE=ddp --force_ddp --graph 0"; do
    envs=$(echo "$spec" | tr ' ' '\n' | grep '=' | grep -v '^--' | tr '\n' ' ')
    args=$(echo "$spec" | tr ' ' '\n' | grep -v '^DCGAN' | tr '\n' ' ')
    r=$(env $envs timeout -k 10 180 python3 bench.py --steps 50 --warmup 10 $args 2>/dev/null) || { echo "failed: $spec" | tee -a $out; exit 1; }
    echo "$spec :: $(echo "$r" | val)" | tee -a $out
  done
done
