"""bench.py --gpus N: the rank launcher and its refusals (CPU, no GPU touched).

The driver runs `bench.py --gpus N` (and torchrun ... bench.py --gpus N); either way N rank
processes must run the data-parallel step (scripts/nerf.py:297-302 sum loss, train_nerf.py:477
loss seed: loma-nerf_amd/dp.py), and the line must never claim n_gpus it did not run. Here the
launcher starts world-size-2 children of a gloo rehearsal script instead of the GPU bench.
"""
import json
import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402  (stdlib-only at import time)


CHILD = textwrap.dedent("""
    import json, os, sys
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    assert r == int(os.environ["RANK"]) == int(os.environ["LOCAL_RANK"]) and w == int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    with open(os.path.join(sys.argv[1], f"rank{r}.json"), "w") as f:
        json.dump({"rank": r, "world": w, "sum": float(t.item()), "argv": sys.argv[2:]}, f)
    dist.destroy_process_group()
""")


def test_launch_ranks_world2_gloo(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    rc = bench.launch_ranks(2, [str(tmp_path), "--steps", "3"], cmd=[sys.executable, str(script)],
                            env={k: v for k, v in os.environ.items() if k not in ("MASTER_PORT", "WORLD_SIZE")})
    assert rc == 0
    got = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    assert [g["rank"] for g in got] == [0, 1]
    assert all(g["world"] == 2 and g["sum"] == 3.0 and g["argv"] == ["--steps", "3"] for g in got)


def test_launch_ranks_propagates_failure(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert bench.launch_ranks(2, [], cmd=[sys.executable, str(script)]) == 3


def test_bench_refuses_world_mismatch():
    """--gpus 2 under a world-size-1 launcher exits non-zero before touching the GPU."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "refusing" in (p.stderr + p.stdout)


def test_variant_labels():
    import argparse
    a = argparse.Namespace(zero_weights=True, generic=False, x6_train=False, k16_w4=False, no_optimizer=False,
                           strong=False, render_k16=False, x6=False, dw_grid=768, input="rays", rays=None,
                           config="cfg3")
    assert bench.variant_flags(a) == ["zero-weights", "dw-grid=768"]
    a = argparse.Namespace(zero_weights=False, generic=False, x6_train=False, k16_w4=False, no_optimizer=False,
                           strong=False, render_k16=False, x6=False, dw_grid=0, input="rays", rays=None,
                           config="cfg3")
    if not os.environ.get("LNERF_LIB"):
        assert bench.variant_flags(a) == []


BLOCKER = textwrap.dedent("""
    import os, sys, time, datetime
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=600))
    if dist.get_rank() == 1:
        sys.exit(5)                      # a rank that dies after the rendezvous
    t = torch.ones(1)
    dist.all_reduce(t)                   # rank 0 blocks here: its peer is gone
    time.sleep(600)
""")


def test_launch_ranks_fails_fast_when_a_peer_dies(tmp_path):
    """rank 1 exits non-zero while rank 0 blocks in all_reduce; the launcher must
    return rank 1's status within ~30 s (it terminates rank 0) instead of waiting for rank 0."""
    import time
    script = tmp_path / "block.py"
    script.write_text(BLOCKER)
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, [], cmd=[sys.executable, str(script)], grace_s=5.0,
                            env={k: v for k, v in os.environ.items() if k not in ("MASTER_PORT", "WORLD_SIZE")})
    took = time.monotonic() - t0
    assert rc == 5
    assert took < 30.0, took
