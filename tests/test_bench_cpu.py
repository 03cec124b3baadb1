"""bench.py's launcher contract, host-only: `--gpus N` without a launcher
starts N ranks itself, a launcher world that differs from --gpus is refused
before anything touches torch or a GPU, and configs[3]'s strong-scaling shard
sizes."""
import os
import subprocess
import sys

import bench
from conftest import REPO


def test_world_check():
    assert bench.world_check(1, {}) is None
    assert bench.world_check(8, {}) == "spawn"
    assert bench.world_check(8, {"WORLD_SIZE": "8"}) is None
    assert bench.world_check(1, {"WORLD_SIZE": "1"}) is None
    assert "WORLD_SIZE=2" in bench.world_check(8, {"WORLD_SIZE": "2"})


def test_world_mismatch_refused_before_torch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    # -X importtime would show torch; simpler: the refusal exits 2 within a
    # second, long before `import torch` could have finished
    p = subprocess.run([sys.executable, "-c",
                        "import sys; sys.argv = ['bench.py', '--gpus', '8']; import bench; bench.main()"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode == 2, p.stderr
    assert "WORLD_SIZE=2 but --gpus 8" in p.stderr


def test_launcher_command():
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "5"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-5:] == [os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "5"]


def test_strong_scaling_shards():
    # configs[3]: the 10 G-base genome split N ways, whole FASTA lines and words
    for n in (1, 2, 4, 8):
        s = bench.shard_bases(10_000_000_000, n, 80)
        assert s * n == 10_000_000_000 and s % 80 == 0 and s % 32 == 0
    s = bench.shard_bases(10_000_000_000, 3, 80)
    assert s % 160 == 0 and 3 * s <= 10_000_000_000
    assert bench.shard_bases(25_600_000, 2, 0) == 12_800_000
