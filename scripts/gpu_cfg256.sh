mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_hip_kernels.py -q -m gpu -x > gpurun_out/k.log 2>&1 || { tail -20 gpurun_out/k.log; exit 1; }
tail -2 gpurun_out/k.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --output_size 256 --batch_size 512 --dtype fp16 > gpurun_out/b256.log 2>&1 || { tail -20 gpurun_out/b256.log; exit 1; }
tail -1 gpurun_out/b256.log
