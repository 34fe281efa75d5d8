"""bench.py's multi-GPU launch (BASELINE metric "at 1/2/4/8 MI355X"): `python bench.py --gpus N` with no launcher
in the environment starts the N rank processes itself (torch.distributed.run as a child, rendezvous on 127.0.0.1)
before anything touches a GPU; under a launcher WORLD_SIZE must equal --gpus.  CPU only: the ranks report their
environment (_BENCH_RANK_PROBE) instead of running the benchmark."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_dry_launch_names_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "7", "--dry-launch"], env=_env(),
                       capture_output=True, text=True, timeout=120, check=True)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["nproc"] == 4 and d["master_addr"] == "127.0.0.1"
    cmd = d["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    i = cmd.index(BENCH)
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "7"]   # the ranks get the same arguments, minus --dry-launch
    assert d["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launch_spawns_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3"], env=_env(_BENCH_RANK_PROBE="1", OMP_NUM_THREADS="1"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(int(d["RANK"]) for d in lines) == [0, 1, 2]
    assert {d["WORLD_SIZE"] for d in lines} == {"3"} and {d["MASTER_ADDR"] for d in lines} == {"127.0.0.1"}
    assert sorted(int(d["LOCAL_RANK"]) for d in lines) == [0, 1, 2]


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], env=_env(WORLD_SIZE="2", _BENCH_RANK_PROBE="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_single_gpu_runs_in_process():
    """N = 1 (the driver's default run) is not relaunched: the process itself is the rank."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=_env(_BENCH_RANK_PROBE="1"),
                       capture_output=True, text=True, timeout=120, check=True)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["WORLD_SIZE"] is None and d["RANK"] is None
