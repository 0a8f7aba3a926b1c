mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -q -m gpu -x > gpurun_out/kernel_tests.log 2>&1; echo "kernel tests rc=$?"; tail -3 gpurun_out/kernel_tests.log
timeout -k 10 600 python benchmarks/bench_kernels.py --batch 128 --write > gpurun_out/kbench.log 2>&1; echo "kbench rc=$?"; cat gpurun_out/kbench.log
mkdir -p gpurun_out/tuned && cp distributed_tensorflow_for_dcgan_amd/ops/igemm_tuned.json gpurun_out/tuned/ 2>/dev/null
true
