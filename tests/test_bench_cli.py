"""bench.py's command-line contract on the CPU (no GPU here): the RCCL
launch refuses more ranks than visible GPUs before any process group exists,
and the BASELINE configs[0] line (the CPU PyTorch path) prints one JSON line."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(args, env_over=None, timeout=300):
    env = dict(os.environ, **(env_over or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_nccl_refuses_more_ranks_than_gpus():
    """WORLD_SIZE=2 under --backend nccl with fewer visible GPUs (none here):
    exit code 3 and a message, before init_process_group (no MASTER_PORT is
    listening, so reaching the rendezvous would hang until the timeout)."""
    r = _run(["--gpus", "2", "--backend", "nccl"],
             dict(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1",
                  HIP_VISIBLE_DEVICES=""), timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "one GPU per rank" in r.stderr


def test_config1_cpu_line():
    """--config 1: the oracle's training step on the host (precrop window,
    TV, RAdam), one JSON line naming BASELINE configs[0]; a reduced batch
    keeps the test short."""
    r = _run(["--config", "1", "--steps", "1", "--n-rand", "64"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert "BASELINE configs[0]" in line["config"]["workload"]
    assert line["n_gpus"] == 0 and line["value"] > 0 and line["unit"] == "rays/s"
