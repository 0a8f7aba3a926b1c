#!/bin/bash
# consumer-side BN-apply VALU proxy (ab_proxy/ build) vs the production igemm3, isolated, per consumer layer
mkdir -p gpurun_out
for r in 1 2; do
  for spec in "G.g_h2.fwd 210:2" "G.g_h3.fwd 211:1" "D2.fwd 210:2" "D3.fwd 213:3"; do
    set -- $spec
    echo "[prod] $(timeout -k 10 120 python -u benchmarks/ig4_study.py --only $1 --ref $2 2>/dev/null | grep cfg)" || exit 1
    echo "[proxy] $(cd ab_proxy && timeout -k 10 120 python -u benchmarks/ig4_study.py --only $1 --ref $2 2>/dev/null | grep cfg)" || exit 1
  done
done | tee gpurun_out/bn_proxy.txt
