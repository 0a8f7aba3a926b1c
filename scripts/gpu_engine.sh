mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -x -q -m gpu > gpurun_out/kernel_tests.log 2>&1; tail -3 gpurun_out/kernel_tests.log
timeout -k 10 600 python -m pytest tests/test_hip_engine.py -q -s -m gpu -k "intermediate or graph or sampler" > gpurun_out/engine_tests.log 2>&1
grep -E "intermediate|^  [dg]|passed|failed|Error|error" gpurun_out/engine_tests.log | head -80
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python bench.py --steps 20 --warmup 3 > gpurun_out/prof2.log 2>&1 || { tail -20 gpurun_out/prof2.log; exit 1; }
tail -1 gpurun_out/prof2.log
