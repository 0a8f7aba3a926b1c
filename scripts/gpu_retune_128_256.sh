#!/bin/bash
./scripts/gpu_retune_cfg.sh "--output_size 128 --steps 60 --warmup 10" "--steps 30 --warmup 5 --output_size 128" r128 && \
./scripts/gpu_retune_cfg.sh "--output_size 256 --batch 512 --dtype fp16 --steps 15 --warmup 3" "--steps 10 --warmup 3 --output_size 256 --batch_size 512 --dtype fp16" r256
