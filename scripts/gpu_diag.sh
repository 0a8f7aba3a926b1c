mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_engine.py -q -s -m gpu > gpurun_out/engine_tests.log 2>&1
grep -E "^  |passed|failed|Error" gpurun_out/engine_tests.log | head -150
