"""CPU: bench.py's multi-rank entry.

``python bench.py --gpus N`` in a plain process must run N ranks: it starts
``torch.distributed.run --nproc-per-node N`` as a child process (no GPU call in the parent,
never an exec), relays rank 0's JSON line and exits with the child's status.  Under a
launcher, an explicit --gpus that disagrees with WORLD_SIZE exits non-zero.  Reference:
train.py:116-120 (init_process_group("nccl")), trainer.py:15-22.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, ROOT)
    import bench as b
    return b


def test_launcher_command(bench):
    cmd = bench.launcher_command(8, ["--gpus", "8", "--steps", "5"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert cmd[-5] == BENCH


def test_check_world(bench):
    assert bench.check_world(None, {}) == (1, None)
    assert bench.check_world(4, {}) == (4, None)
    assert bench.check_world(None, {"WORLD_SIZE": "2"}) == (2, None)
    assert bench.check_world(2, {"WORLD_SIZE": "2"}) == (2, None)
    world, err = bench.check_world(8, {"WORLD_SIZE": "2"})
    assert world == 2 and err is not None and "--gpus 8" in err


def test_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=3" in r.stderr
    assert r.stdout == ""


def test_launch_relays_child_output_and_status(bench, monkeypatch, capsys):
    """The child's stdout (rank 0's JSON line) is relayed; its exit code is returned."""
    script = "import sys; print('{\"metric\": \"x\", \"n_gpus\": %d}' % int(sys.argv[1])); sys.exit(3)"
    monkeypatch.setattr(bench, "launcher_command", lambda n, argv, port: [sys.executable, "-c", script, str(n)])
    rc = bench.launch_ranks(4, [])
    assert rc == 3
    assert capsys.readouterr().out.strip() == '{"metric": "x", "n_gpus": 4}'


def test_torchrun_two_ranks_env():
    """The real launcher with a stand-in rank program: 2 ranks, each sees WORLD_SIZE=2 and a
    distinct RANK/LOCAL_RANK; only rank 0 prints."""
    code = ("import os, json\n"
            "if os.environ['RANK'] == '0':\n"
            "    print(json.dumps({'world': os.environ['WORLD_SIZE'], 'local': os.environ['LOCAL_RANK'], "
            "'addr': os.environ['MASTER_ADDR']}))\n")
    sys.path.insert(0, ROOT)
    import bench as b
    prog = os.path.join(ROOT, "tests", "_rank_probe_tmp.py")
    with open(prog, "w") as f:
        f.write(code)
    try:
        cmd = b.launcher_command(2, [], b.free_port())
        cmd[cmd.index(BENCH)] = prog
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    finally:
        os.remove(prog)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == '{"world": "2", "local": "0", "addr": "127.0.0.1"}'
