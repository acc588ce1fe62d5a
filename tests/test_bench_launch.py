"""CPU: `python bench.py --gpus N` without a launcher starts N ranks itself (one process per
GPU, as the driver's torchrun runs do) and refuses a rank count that differs from --gpus."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_logic():
    assert bench.needs_launch(2, False, {})
    assert bench.needs_launch(8, False, {"RANK": "0"})
    assert not bench.needs_launch(1, False, {})
    assert not bench.needs_launch(2, True, {})                   # one process drives the devices
    assert not bench.needs_launch(2, False, {"WORLD_SIZE": "2"})  # already a rank of a launch
    cmd = bench.worker_command(["--gpus", "2", "--steps", "5"], 2, 29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "2"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "2", "--steps", "5"] and cmd[-5].endswith("bench.py")
    bench.check_world(2, 2, False)
    bench.check_world(2, 1, True)
    with pytest.raises(SystemExit):
        bench.check_world(2, 1, False)


def test_gpus_two_starts_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert {x["world"] for x in lines} == {2} and sorted(x["local_rank"] for x in lines) == [0, 1]


def test_rank_count_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_parity_mismatch_fails_the_run(capsys):
    """A bench line whose results differ from the oracle is still printed, but the run exits
    non-zero (bench.report is what main() and bench_order() return to sys.exit)."""
    out = {"metric": "m", "value": 1.0, "parity": "MISMATCH vs C oracle"}
    assert bench.report(out, False) == bench.PARITY_EXIT != 0
    line = capsys.readouterr().out.strip()
    assert json.loads(line)["parity"] == "MISMATCH vs C oracle"
    assert bench.report(dict(out, parity="bit-exact"), True) == 0
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "return report(out, parity_ok)" in src and "return report(out, parity)" in src
    assert "sys.exit(main())" in src


def test_stage_layout_names_every_event():
    """The timing-mode stages the bench line reports at each shape."""
    base = ["k_pod_reduce", "k_step_tail", "k_order_split"]
    assert bench.stage_layout(1, 1, None, "nccl") == base + ["k_node_groups"]
    assert bench.stage_layout(1, 8, None, "nccl") == base + ["k_node_groups+decide"]            # --shard-of 8
    assert bench.stage_layout(8, 8, None, "nccl") == base + ["exchange", "k_node_groups+decide"]
    assert bench.stage_layout(2, 2, None, "gloo") == base + ["exchange_host_staged", "k_node_groups+decide"]
    assert bench.stage_layout(1, 1, [0, 1], "multi") == base + ["exchange", "k_node_groups+decide"]


def test_rccl_ranks_field_is_truthful():
    """`rccl_ranks` is ncclCommCount of a live communicator, never a device count: None for a
    multi-device context on its peer exchange (esc_comm_size 0), for gloo and for one rank."""
    def never():
        raise AssertionError("no communicator to ask")
    assert bench.rccl_ranks_field(lambda: 0, [0, 0], 1, "multi") is None          # peer exchange
    assert bench.rccl_ranks_field(lambda: 2, [0, 1], 1, "multi") == 2             # ncclCommInitAll
    assert bench.rccl_ranks_field(lambda: 8, None, 8, "nccl") == 8
    assert bench.rccl_ranks_field(never, None, 2, "gloo") is None
    assert bench.rccl_ranks_field(never, None, 1, "nccl") is None
