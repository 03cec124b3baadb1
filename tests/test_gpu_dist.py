"""Sharded multi-process path on the GPU box: bench.py under torchrun with
two ranks sharing cuda:0 and host-side (gloo) collectives.  Exercises the
real engine's feed_shard / summary / resolve / table exchange through
findkmer_amd/dist.py; bench.py asserts the merged table and the summed
window counts against the exact totals of the one stream.  (RCCL itself
needs one GPU per rank: the driver's multi-GPU bench covers it.)"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("k,fasta,chrom", [(6, 0, 1_500_000_000), (11, 80, 1_500_000_000), (6, 0, 20_000_000),
                                           (7, 0, 12_799_900)])
def test_two_rank_shards_gloo(k, fasta, chrom):
    """chrom < 25.6M puts an 'N' run break inside rank 1's shard (20M), or in
    its 256-byte halo (12_799_900: 100 bases before the shard)"""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(29600 + k + chrom % 97), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dist-backend", "gloo",
           "--k", str(k), "--fasta-line", str(fasta), "--bases", "12800000", "--chrom", str(chrom)]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["value"] > 0
