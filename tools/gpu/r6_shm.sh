#!/bin/bash
# GPU box: N-rank data-parallel tests on one GPU through the /dev/shm stand-in
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dp_shm.py -x -v --timeout 600 --timeout-method thread > gpurun_out/shm_tests.log 2>&1
rc=$?
tail -40 gpurun_out/shm_tests.log
exit $rc
