"""bench.py's multi-GPU self-launch: `python bench.py --gpus N` with no
torch.distributed environment starts N ranks as a child `torch.distributed.run`, never
falls back to one rank, and refuses N above the visible devices.  CPU-only: the decision
and the command line are checked here; the child run itself is the GPU rehearsal."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_single_gpu_runs_inline():
    assert bench.launch_plan(1, {}, 0, ["--gpus", "1"]) == ("inline", None)


def test_rank_of_a_launch_runs_inline():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    assert bench.launch_plan(8, env, 8, ["--gpus", "8"]) == ("inline", None)


def test_world_size_mismatch_is_an_error():
    act, msg = bench.launch_plan(8, {"WORLD_SIZE": "4"}, 8, [])
    assert act == "error" and "WORLD_SIZE=4" in msg


def test_spawns_torchrun_child_with_all_arguments():
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    act, cmd = bench.launch_plan(8, {}, 8, argv, port=31337)
    assert act == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "31337"
    assert cmd[-len(argv) - 1] == str(ROOT / "bench.py") and cmd[-len(argv):] == argv


def test_too_few_devices_is_an_error_not_one_rank():
    act, msg = bench.launch_plan(8, {}, 1, ["--gpus", "8"])
    assert act == "error" and "only 1" in msg


def test_rehearsal_allows_ranks_on_one_device():
    act, cmd = bench.launch_plan(2, {"C3H_BENCH_REHEARSAL": "1"}, 1, ["--gpus", "2"])
    assert act == "spawn" and cmd[cmd.index("--nproc-per-node") + 1] == "2"


def test_child_env_marks_child_and_keeps_dmabuf_ipc():
    env = bench.child_env({"PATH": "/bin"})
    assert env["C3H_BENCH_CHILD"] == "1" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_relay_keeps_only_the_result_line_on_stdout():
    import io
    script = ("import json, sys; print('[Gloo] Rank 0 is connected to 1 peer ranks'); "
              "print(json.dumps({'metric': 'm', 'value': 1.0})); print('{not json'); sys.exit(3)")
    out, err = io.StringIO(), io.StringIO()
    rc = bench.relay([sys.executable, "-c", script], None, out=out, err=err)
    assert rc == 3
    assert out.getvalue().splitlines() == ['{"metric": "m", "value": 1.0}']
    assert "[Gloo]" in err.getvalue() and "{not json" in err.getvalue()


def test_bench_exits_nonzero_without_devices():
    """This container has no HIP device: --gpus 2 must fail loudly, not run one rank."""
    env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "C3H_BENCH_REHEARSAL")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "--gpus 2 requested but only 0" in r.stderr
    assert r.stdout.strip() == ""
