"""bench.py's own rank launcher (a bare `python bench.py --gpus N`): N rank processes over a 127.0.0.1 rendezvous,
started before anything touches the GPU.  --dry-launch brings the ranks up over gloo without a GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bare_bench_launches_its_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-launch"], env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # only rank 0 prints
    rec = json.loads(lines[0])
    assert rec["world"] == 2
    assert sorted(r["rank"] for r in rec["ranks"]) == [0, 1]
    assert sorted(r["local_rank"] for r in rec["ranks"]) == [0, 1]
    assert len({r["pid"] for r in rec["ranks"]}) == 2


def test_launcher_propagates_a_failing_rank():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["BENCH_DRY_FAIL_RANK"] = "1"  # rank 1 dies before the rendezvous; rank 0 would wait for it forever
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-launch"], env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 3
