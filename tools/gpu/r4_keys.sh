#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
true

timeout -k 10 200 python -u tools/gpu/keys.py c5 20 > gpurun_out/keys_c5.txt 2> gpurun_out/keys_c5.err || { tail gpurun_out/keys_c5.err; exit 1; }
cat gpurun_out/keys_c5.txt
timeout -k 10 200 python -u tools/gpu/keys.py c3 20 > gpurun_out/keys_c3.txt 2> gpurun_out/keys_c3.err || { tail gpurun_out/keys_c3.err; exit 1; }
cat gpurun_out/keys_c3.txt
