"""bench.py's multi-GPU plumbing on CPU (gloo): `--gpus N` without torchrun
starts N fresh ranks itself, times with barrier + max over ranks and prints
one line on rank 0; a rank count that disagrees with --gpus is an error.
(--cpu-dry-run swaps the GPU work for a rank-dependent sleep.)"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=e, capture_output=True, text=True,
                          timeout=240)


def test_gpus_n_spawns_n_ranks_and_aggregates():
    p = run(["--gpus", "2", "--steps", "5", "--warmup", "1", "--frames", "1000", "--cpu-dry-run"])
    assert p.returncode == 0, p.stderr
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 5 and d["scaling"] == "weak"
    assert [r["rank"] for r in d["per_gpu"]] == [0, 1]
    # rank 1 sleeps twice as long per step: the job time is the slowest rank's
    assert d["per_gpu"][1]["Mpkt_s"] < d["per_gpu"][0]["Mpkt_s"]
    assert abs(d["value"] - 2 * d["per_gpu"][1]["Mpkt_s"]) / d["value"] < 0.35
    # every rank describes itself: its roofline kernel's
    # time and fraction, its staging-probe outcome, its GPU
    for r in d["per_gpu"]:
        for k in ("decode_ms", "decode_alg_bytes", "decode_frac", "staging_probe", "bdf"):
            assert k in r, (k, r)
        assert "chosen" in r["staging_probe"] and "ns_per_frame" in r["staging_probe"]
    agg = d["roofline_all_gpus"]
    # sum of the ranks' bytes over the slowest rank's time, against N x 8 TB/s
    alg = sum(r["decode_alg_bytes"] for r in d["per_gpu"])
    t = max(r["decode_ms"] for r in d["per_gpu"]) * 1e-3
    assert agg["peak"] == 2 * 8000.0 and abs(agg["frac"] - alg / t / 1e9 / 16000.0) < 1e-3
    assert agg["slowest_rank"] == 1 and agg["min_rank_frac"] == d["per_gpu"][1]["decode_frac"]


def test_default_is_one_rank():
    p = run(["--steps", "3", "--frames", "1000", "--cpu-dry-run"])
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["per_gpu"] is None


def test_world_size_mismatch_is_an_error():
    p = run(["--gpus", "1", "--steps", "2", "--cpu-dry-run"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_rehearsal():
    """The N-rank bench on hardware: `--gpus 2` starts two ranks that each
    run their own queue on the GPU (shared here: one-GPU box, control plane
    over gloo), barrier + max over ranks, one line from rank 0."""
    p = run(["--gpus", "2", "--share-gpu", "--steps", "3", "--warmup", "1", "--frames", "65536", "--no-9000",
             "--no-cpu-baseline"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and [r["rank"] for r in d["per_gpu"]] == [0, 1]
    assert all(r["Mpkt_s"] > 0 for r in d["per_gpu"])
    assert "shared-GPU rehearsal" in d["config"]["parallelism"]
