"""The bench contract line (bench.py compact_line): the driver parses the ONE
stdout JSON line; round 5's 26.8 KB line came back unparsed.  Built here from
recorded full records (profiles/r4, profiles/r5 bench_default.json, the shape
bench.py's `out` dict has), the line must hold every contract key, the full
roofline and cpu_baseline, and stay under CONTRACT_LINE_MAX bytes."""
import copy
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORDS = [os.path.join(ROOT, "profiles", r, "bench_default.json") for r in ("r4", "r5")]


@pytest.mark.parametrize("path", RECORDS, ids=["r4", "r5"])
def test_contract_line_from_recorded_record(path):
    full = json.load(open(path))
    line = json.dumps(bench.compact_line(full))
    assert len(line) <= bench.CONTRACT_LINE_MAX
    c = json.loads(line)
    for k in bench.CONTRACT_KEYS:
        assert k in c, k
    assert c["roofline"] == full["roofline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert c["cpu_baseline"][k] == full["cpu_baseline"][k]
    assert "dropped" not in c      # a recorded default run fits without dropping anything
    # the compact summaries the review asks for
    c5 = c["c5_bf16"]
    assert c5["roofline"]["frac"] == full["c5_bf16"]["roofline"]["frac"]
    for blk in (c["projected_scaling"], c5["projected_scaling"]):
        for mode in ("weak", "strong"):
            for n in ("2", "4", "8"):
                row = blk[mode][n]
                assert {"step_ms", "exposed_exchange_us", "speedup", "step_mode"} <= set(row)
    assert c["small_batch"]["value"] == full["small_batch"]["value"]
    assert "kernels_by_phase" not in line


def test_contract_line_drops_optional_blocks_to_fit():
    full = json.load(open(RECORDS[-1]))
    big = copy.deepcopy(full)
    big["c5_bf16"]["workload"] = "x" * 20000          # an oversize optional block
    c = bench.compact_line(big)
    line = json.dumps(c)
    # contract keys survive; the oversize block is dropped and named
    for k in bench.CONTRACT_KEYS:
        assert k in c
    assert c["dropped"]
    assert len(line) <= bench.CONTRACT_LINE_MAX and "c5_bf16" in c["dropped"]


def test_contract_line_world_gt_1_shape():
    """An N > 1 rank-0 record (no projections, no small batch, cpu_baseline
    None, an exchange table) still yields the contract keys."""
    full = json.load(open(RECORDS[-1]))
    for k in ("projected_scaling", "small_batch"):
        full.pop(k)
    full["c5_bf16"].pop("projected_scaling")
    full["cpu_baseline"] = None
    full["n_gpus"] = 8
    full["exchange"] = {"rccl_allreduce": {"avg_us": 50.0, "per_step": 4, "MB_per_step": 13.2}}
    c = bench.compact_line(full)
    assert len(json.dumps(c)) <= bench.CONTRACT_LINE_MAX
    assert c["cpu_baseline"] is None and c["exchange"] == full["exchange"]


_GLOO_CHILD = r"""
import os, sys
sys.path.insert(0, %r)
import bench
import torch.distributed as dist
with bench.stdout_to_stderr():
    dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=2)
dist.barrier()
dist.destroy_process_group()
"""


def test_gloo_init_keeps_stdout_clean(tmp_path):
    """bench.py's N > 1 ranks init their gloo group inside stdout_to_stderr:
    Gloo prints a peer-connection line on fd 1 at init, which would put a
    second line beside the contract's one JSON line (found rehearsing the
    N-rank bench on one GPU, tools/gpu/r6_rehearse.sh)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = tmp_path / "child.py"
    src.write_text(_GLOO_CHILD % root)
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT="29671")
        procs.append(subprocess.Popen([sys.executable, str(src)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, cwd=root))
    outs = [p.communicate(timeout=120) for p in procs]
    assert [p.returncode for p in procs] == [0, 0], [o[1][-500:] for o in outs]
    assert all(o[0] == b"" for o in outs), [o[0][:200] for o in outs]
