#!/bin/bash
# GPU box: the forward-layer pack -- its bitwise tests, then same-box A/B
# (A = pack, the default; B = DDPG_FWD_PACK=0) at C3 and C5
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu tests/test_gpu_switches.py -k "fwd_pack or gemm_pack" -x -q --timeout 300 --timeout-method thread > gpurun_out/fwdpack_tests.log 2>&1 || { tail -30 gpurun_out/fwdpack_tests.log; exit 1; }
tail -2 gpurun_out/fwdpack_tests.log
bash tools/gpu/envab.sh DDPG_FWD_PACK=0 c3 3 gemm || exit $?
bash tools/gpu/envab.sh DDPG_FWD_PACK=0 c5 3 gemm || exit $?
