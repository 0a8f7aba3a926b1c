#!/bin/bash
# final-tree check of the live single-GPU knobs' defaults (interleaved x3, 200/20)
./scripts/gpu_ab_vals.sh DCGAN_NCONV_CAP "512 1024 256" && ./scripts/gpu_ab_vals.sh DCGAN_IGEMM_LPT "1 0"
