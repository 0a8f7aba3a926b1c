set -e
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.is_available(), torch.cuda.get_device_name(0))"
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -x -q -m gpu > gpurun_out/kernels.log 2>&1 || { tail -50 gpurun_out/kernels.log; exit 1; }
tail -5 gpurun_out/kernels.log
timeout -k 10 300 python bench.py --engine reference --steps 20 --warmup 5 > gpurun_out/bench_ref.log 2>&1
tail -2 gpurun_out/bench_ref.log
