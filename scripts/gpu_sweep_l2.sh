#!/bin/bash
# stand-in bandwidth / wire sweep, then the L2 hit-rate counter pass
./scripts/gpu_standin_sweep.sh && ./scripts/gpu_pmc_l2.sh
