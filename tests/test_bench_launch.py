"""bench.py's launch logic on the CPU (no GPU): the launcher-less N-rank spawn (spawn_ranks) and the
WORLD_SIZE / --gpus consistency check. The spawned "ranks" here are tiny stand-in scripts, so only the
process handling is exercised: environment, rank-0 JSON forwarding, failure propagation."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run_spawn(tmp_path, monkeypatch, capsys, body, n):
    import bench
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(body))
    monkeypatch.setattr(bench, "__file__", str(script))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", str(n)])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    rc = bench.spawn_ranks(n)
    return rc, capsys.readouterr()


def test_spawn_ranks_environment_and_rank0_line(tmp_path, monkeypatch, capsys):
    rc, out = _run_spawn(tmp_path, monkeypatch, capsys, """
        import json, os, sys
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GLS_BENCH_SPAWNED")
        env = {k: os.environ.get(k) for k in keys}
        print("progress line of rank", env["RANK"])
        if env["RANK"] == "0":
            print(json.dumps({"metric": "m", "env": env, "argv": sys.argv[1:]}))
        """, 3)
    assert rc == 0
    lines = [l for l in out.out.splitlines() if l.strip()]
    assert len(lines) == 1, out.out  # exactly one line on stdout: rank 0's JSON
    rec = json.loads(lines[0])
    env = rec["env"]
    assert env["RANK"] == "0" and env["LOCAL_RANK"] == "0" and env["WORLD_SIZE"] == "3"
    assert env["MASTER_ADDR"] == "127.0.0.1" and int(env["MASTER_PORT"]) > 0 and env["GLS_BENCH_SPAWNED"] == "1"
    assert rec["argv"] == ["--gpus", "3"]
    assert "progress line of rank 0" in out.err


def test_spawn_ranks_failure_terminates_the_others(tmp_path, monkeypatch, capsys):
    rc, out = _run_spawn(tmp_path, monkeypatch, capsys, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(7)
        time.sleep(120)  # rank 0 would wait forever for its peer
        """, 2)
    assert rc == 7
    assert "terminating the others" in out.err
    assert out.out.strip() == ""


def test_spawn_ranks_no_result_line_is_an_error(tmp_path, monkeypatch, capsys):
    rc, _ = _run_spawn(tmp_path, monkeypatch, capsys, "print('no json here')\n", 2)
    assert rc == 1


@pytest.mark.parametrize("world,gpus", [("2", 1), ("4", 8), ("1", 2)])
def test_world_size_must_match_gpus(world, gpus):
    env = dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--no-cpu"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 1, out.stderr
    assert "WORLD_SIZE=%s but --gpus %d" % (world, gpus) in out.stderr
    assert out.stdout.strip() == ""


def _agree_worker(rank, world, port, failed, late, stuck, q):
    import datetime

    import torch.distributed as dist

    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctl = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=5))
    if stuck[rank]:  # never reaches the agreement (a rank left inside a data-path collective)
        import time
        time.sleep(12)
        q.put((rank, "stuck"))
        return
    q.put((rank, bench.preflight_agreement(dist, ctl, world, failed[rank], late[rank])))


@pytest.mark.parametrize("failed,late,stuck,want", [
    ((False, False), (False, False), (False, False), {0: "ok", 1: "ok"}),
    ((False, True), (False, False), (False, False), {0: "fallback", 1: "fallback"}),  # before the first collective
    ((True, True), (True, True), (False, False), {0: "fallback", 1: "fallback"}),     # every rank failed: none stuck
    ((False, True), (False, True), (False, False), {0: "abort", 1: "abort"}),         # rank 1 only, after it
    ((False, True), (False, True), (True, False), {1: "abort"}),                      # rank 0 never arrives
])
def test_preflight_agreement_over_the_control_group(failed, late, stuck, want):
    """the native transport falls back to torch.distributed only when no rank can be inside one of
    its collectives; the ranks agree over a gloo group with a timeout, so a rank whose peer is stuck aborts
    instead of hanging (gloo, world size 2, CPU)."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_agree_worker, args=(r, 2, port, failed, late, stuck, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=90) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    for r, v in want.items():
        assert got[r] == v, got
