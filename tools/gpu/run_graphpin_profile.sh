#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph_pin.py tests/test_gpu_configs.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/gputests2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/gputests2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu/profile.sh c3
