"""bench.py's --gpus / WORLD_SIZE contract (no GPU: --launch-check reports each rank's environment and exits
before any HIP call).  Without a launcher, --gpus N > 1 must start N ranks itself (CommandStores.mapReduce's
per-store fan-out, accord-core/src/main/java/accord/local/CommandStores.java:576-593); under a launcher a
WORLD_SIZE that differs from --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=120)


def test_gpus_n_spawns_n_ranks():
    r = run(["--gpus", "3", "--launch-check"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout                     # only rank 0's line reaches stdout
    rec = json.loads(lines[0])
    assert rec["rank"] == 0 and rec["world"] == 3 and rec["gpus"] == 3
    assert rec["master"].startswith("127.0.0.1:")
    for k in (1, 2):
        assert "rank %d of 3 (local %d)" % (k, k) in r.stderr


def test_single_gpu_runs_in_process():
    r = run(["--gpus", "1", "--launch-check"])
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip())
    assert rec["world"] == 1 and rec["rank"] == 0


def test_world_size_mismatch_refused():
    r = run(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"}, drop=())
    assert r.returncode != 0
    assert "WORLD_SIZE=4" in r.stderr
    r = run(["--launch-check"], {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"}, drop=())
    assert r.returncode != 0                             # default --gpus 1 under an 8-rank launcher


def test_launcher_world_matches():
    r = run(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0",
                                                 "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29999"}, drop=())
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip())
    assert rec["world"] == 2 and rec["rank"] == 0      # the launcher's rank runs itself, nothing spawned


def test_failing_rank_fails_the_job():
    # a rank that cannot start (bad argument parsed by every child) makes the whole job exit non-zero
    r = run(["--gpus", "2", "--launch-check", "--config", "C9"])
    assert r.returncode != 0
