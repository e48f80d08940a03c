#!/bin/bash
# GPU box: the gemm_h256 GPU tests, then the DDPG_GEMM256 A/B at C5 ($1 values)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_switches.py::test_gemm256_switch_bf16" "tests/test_gpu_configs.py::test_c5_bf16_full_dims" \
  > gpurun_out/g256tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|^E " gpurun_out/g256tests.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NOTESTS=1 bash tools/gpu/gemm256_ab.sh "$1"
