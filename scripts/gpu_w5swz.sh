#!/bin/bash
# wgrad5 window swizzle for 8-wide outputs: tests + A/B vs ab_old, then the step PMC table
./scripts/gpu_ab_so.sh "wgrad5" && OUT=step_pmc_w5.txt ./scripts/gpu_pmc_step.sh
