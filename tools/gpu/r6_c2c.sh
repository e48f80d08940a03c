#!/bin/bash
# GPU box: a bitwise-neutral small-path change vs tools/abr6/libA.so -- bitwise
# comparison (B = 64, 50, 256), the small-path GPU tests, same-box C2
# latency, kernel trace of the new build
mkdir -p gpurun_out
cp distributed_ddpg_amd/libddpg_hip.so tools/abr6/libB.so
T="timeout -k 10"
$T 180 python -u tools/gpu/c2_bitwise.py new || exit $?
DDPG_LIB_PATH=tools/abr6/libA.so $T 180 python -u tools/gpu/c2_bitwise.py old || exit $?
python tools/gpu/c2_bitwise.py --cmp old new
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_graph_pin.py tests/test_gpu_dp.py tests/test_gpu_dp_shm.py > gpurun_out/c2_tests.log 2>&1 || { tail -30 gpurun_out/c2_tests.log; exit 1; }
tail -2 gpurun_out/c2_tests.log
for r in 1 2 3; do
  for v in A B; do
    DDPG_LIB_PATH=tools/abr6/lib$v.so $T 120 python -u tools/gpu/c2_sync.py $v || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2prof -o run -- python3 bench.py --config c2 --no-cpu --no-small --no-project --steps 200 --warmup 20 > gpurun_out/c2prof.json 2> gpurun_out/c2prof.err || exit $?
python3 profiles/summarize.py gpurun_out/c2prof/run_results.db | grep -A6 "per-grid"
