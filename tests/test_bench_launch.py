"""CPU: bench.py's multi-rank launch (`--gpus N` without torchrun) and the push rules.

`python bench.py --gpus 2 --dry-run` must start two rank processes itself (RANK / WORLD_SIZE set,
rendezvous on 127.0.0.1), they join a gloo group, and rank 0 prints one JSON line naming both
ranks. The GPU path uses the same launcher with RCCL (`--gpus` used to be ignored).
"""
import json
import os
import subprocess
import sys
import tarfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    line = _run(["--gpus", "2", "--dry-run"])
    assert line["dry_run"] is True and line["n_gpus"] == 2
    assert [r["rank"] for r in line["ranks"]] == [0, 1]
    assert [r["local_rank"] for r in line["ranks"]] == [0, 1]


def test_bench_gpus1_is_one_process():
    line = _run(["--dry-run"])
    assert line["n_gpus"] == 1 and [r["rank"] for r in line["ranks"]] == [0]


def test_reference_build_does_not_travel(tmp_path):
    """.gpurunignore keeps oracle/_ref (the reference's ctree compiled here) out of every push:
    checked with tar's own --exclude-from semantics on a scratch tree of the same layout."""
    pats = [ln.strip() for ln in open(os.path.join(REPO, ".gpurunignore")) if ln.strip() and not ln.startswith("#")]
    assert "./oracle/_ref" in pats
    root = tmp_path / "repo"
    for rel in ("oracle/_ref/mz_tree.cpython-310-x86_64-linux-gnu.so", "oracle/liblzoracle.so",
                "lightzero_amd/liblzmcts.so", "oracle/lz_oracle.c"):
        f = root / rel
        f.parent.mkdir(parents=True, exist_ok=True)
        f.write_bytes(b"x")
    out = tmp_path / "push.tar"
    subprocess.check_call(["tar", "-cf", str(out), "--exclude-from", os.path.join(REPO, ".gpurunignore"), "."],
                          cwd=root)
    names = tarfile.open(out).getnames()
    assert not any("_ref" in n for n in names), names
    for keep in ("./oracle/liblzoracle.so", "./lightzero_amd/liblzmcts.so", "./oracle/lz_oracle.c"):
        assert keep in names, (keep, names)
