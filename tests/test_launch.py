"""The reference's launch contract without a GPU (ddpg.py:162-174,
parameters.py:32-33): one `--job_name=ps` process hosts the rendezvous and two
`--job_name=worker --task_index=i` processes join it, form the gloo group and
exchange the 128-byte communicator id exactly as learner.init_comm does
(--rendezvous_only stops there: RCCL itself needs the GPUs)."""
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_ps_and_two_workers_rendezvous():
    port = _free_port()
    ps_addr = "127.0.0.1:%d" % port
    workers = "127.0.0.1:%d,127.0.0.1:%d" % (_free_port(), _free_port())
    env = dict(os.environ, PYTHONPATH=ROOT)
    base = [sys.executable, "-m", "distributed_ddpg_amd.ddpg", "--ps", ps_addr, "--workers",
            workers]
    ps = subprocess.Popen(base + ["--job_name=ps", "--task_index=0"], cwd=ROOT, env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        time.sleep(1.0)
        ws = [subprocess.Popen(base + ["--job_name=worker", "--task_index=%d" % i,
                                       "--rendezvous_only"], cwd=ROOT, env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
              for i in range(2)]
        outs = [w.communicate(timeout=120)[0] for w in ws]
        for w, o in zip(ws, outs):
            assert w.returncode == 0, o
        lines = [[l for l in o.splitlines() if l.startswith("rendezvous ok")][0] for o in outs]
        assert "rank 0 of 2" in lines[0] and "rank 1 of 2" in lines[1], lines
        assert lines[0].split()[-1] == lines[1].split()[-1], lines  # same id on both ranks
        assert ps.poll() is None  # the ps blocks like server.join()
    finally:
        ps.kill()
        ps.wait()
