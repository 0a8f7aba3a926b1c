#!/bin/bash
# round 6: D-backward merge timing prototype (heuristic tiles, then the 2B dgrads' tiles)
mkdir -p gpurun_out
{ timeout -k 10 300 python -u benchmarks/study/dmerge_proto.py --rounds 3 --steps 200 --warmup 20 --tiles heur || exit 1
  timeout -k 10 300 python -u benchmarks/study/dmerge_proto.py --rounds 3 --steps 200 --warmup 20 --tiles same2b || exit 1
  timeout -k 10 300 python -u benchmarks/study/dmerge_proto.py --rounds 3 --steps 20 --warmup 5 --tiles same2b || exit 1
} 2>&1 | tee gpurun_out/dmerge_proto_r6.txt
