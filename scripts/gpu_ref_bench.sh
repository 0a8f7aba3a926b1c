set -e
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.is_available(), torch.cuda.get_device_name(0))"
timeout -k 10 300 python bench.py --engine reference --steps 20 --warmup 5 > gpurun_out/bench_ref.log 2>&1
cat gpurun_out/bench_ref.log | tail -2
