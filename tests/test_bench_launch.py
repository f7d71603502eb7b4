"""CPU: `bench.py --gpus N` launches N workers itself (torch.distributed.run as a child, gloo for
the self-test) and refuses a world size that does not match --gpus."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=timeout, cwd=str(ROOT))


def test_self_launch_two_workers_cover_every_chunk_once():
    r = _run(["--gpus", "2", "--launcher-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["world"] == 2 and line["max_rank"] == 1.0
    ranks = sorted(line["ranks"])
    assert [p[0] for p in ranks] == [0, 1] and all(p[1] == 2 for p in ranks)
    # C3: the fixed 256-chunk table and C5: the 92 lineitem chunks, each split contiguously
    assert ranks[0][2] == 0 and ranks[0][3] == ranks[1][2] and ranks[1][3] == 256
    assert ranks[0][4] == 0 and ranks[0][5] == ranks[1][4] and ranks[1][5] == 92
    assert ranks[0][3] == 128  # equal chunks -> an even split


def test_world_mismatch_exits_nonzero():
    r = _run(["--gpus", "1", "--launcher-selftest"], env={"WORLD_SIZE": "2", "RANK": "0"}, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
