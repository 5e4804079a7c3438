"""CPU: bench.py's rank fan-out.  `python bench.py --gpus 2`
without a launcher starts two ranks itself; a launcher whose WORLD_SIZE
differs from --gpus is an error.  MPLIB_AMD_BENCH_DRYRUN=1 runs the launch,
process group (gloo), barrier and max-over-ranks reduction without device
work (no GPU here); the -m gpu twin is test_bench_one_rank_nccl."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env.update(kw)
    return env


def test_bench_gpus2_spawns_two_ranks():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                          "--warmup", "0"], env=_env(MPLIB_AMD_BENCH_DRYRUN="1", MPLIB_AMD_DIST_BACKEND="gloo"),
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["dry_run"] and r["max_rank"] == 1 and r["backend"] == "gloo"


def test_bench_world_size_mismatch_fails():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                         env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MPLIB_AMD_BENCH_DRYRUN="1"),
                         capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr
