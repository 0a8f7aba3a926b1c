#!/bin/bash
./scripts/gpu_r6_f.sh && ./scripts/gpu_r6_g.sh
