#!/bin/bash
# GPU box: round-over-round same-box comparison, R4 = the round-4 head (c6202fc), R5 = this round's head
mkdir -p gpurun_out
bash tools/gpu/ab.sh c3 3 && bash tools/gpu/ab.sh c5 2
