#!/bin/bash
# GPU box: the tests added late in round 6
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu tests/test_gpu_dp_shm.py tests/test_gpu_parity.py tests/test_gpu_switches.py -k "shm or widea or state_half" -x -v --timeout 600 --timeout-method thread > gpurun_out/new_tests.log 2>&1
rc=$?
tail -30 gpurun_out/new_tests.log
exit $rc
