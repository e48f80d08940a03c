#!/bin/bash
# GPU box: rehearse the driver's N-rank bench command with 2 ranks on the one
# GPU (the /dev/shm stand-in for RCCL, eager steps): bench.py's own rank
# spawning and torch.distributed.run, every leg (C3, C5 bf16, C2 + per-rank)
mkdir -p gpurun_out
export DDPG_LIB_PATH=tools/shm/libddpg_shm.so DDPG_GRAPH_COMM=0 DDPG_BENCH_ONE_DEVICE=1
timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu > gpurun_out/reh_spawn.json 2> gpurun_out/reh_spawn.err || { tail -20 gpurun_out/reh_spawn.err; exit 1; }
wc -c gpurun_out/reh_spawn.json
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu > gpurun_out/reh_torchrun.json 2> gpurun_out/reh_torchrun.err || { tail -20 gpurun_out/reh_torchrun.err; exit 1; }
wc -c gpurun_out/reh_torchrun.json
python3 - <<'PY'
import json
for f in ("gpurun_out/reh_spawn.json", "gpurun_out/reh_torchrun.json"):
    lines = [l for l in open(f) if l.strip()]
    d = json.loads(lines[-1])
    print(f, len(lines), "line(s):", d["n_gpus"], d["value"], d["ms_per_step"], d["scaling"],
          "c5", (d.get("c5_bf16") or {}).get("value"), "c2", (d.get("small_batch") or {}).get("value"),
          "dropped", d.get("dropped"))
PY
