#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/thin_k_bench > gpurun_out/tk_c128.txt 2>&1 && timeout -k 10 120 ./tools/thin_k_bench_c64 > gpurun_out/tk_c64.txt 2>&1 || { tail gpurun_out/tk_c64.txt; exit 1; }
for f in tk_c128 tk_c64; do echo "== $f"; grep -A40 "8 row tiles" gpurun_out/$f.txt | grep -A1 "5 parts twin-only"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pack_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pack_tests.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pack_tests.log | head -20; tail -30 gpurun_out/pack_tests.log; exit $rc; }
timeout -k 10 200 python -u tools/gpu/keys.py c5 20 > gpurun_out/keys_c5_pack.txt 2> gpurun_out/keys_c5_pack.err || { tail gpurun_out/keys_c5_pack.err; exit 1; }
head -12 gpurun_out/keys_c5_pack.txt; tail -1 gpurun_out/keys_c5_pack.txt
bash tools/gpu/envab.sh DDPG_GEMM_PACK=0 c5 2 gemm_h16i 2>&1 | tee gpurun_out/pack_ab_c5.txt
