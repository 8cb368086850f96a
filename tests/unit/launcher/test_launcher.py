"""Launcher (reference `tests/unit/launcher/test_run.py`, `test_multinode_runner.py`): hostfile parsing,
include/exclude filters, world-info round trip, per-node rank environments, and a real 2-process local launch."""
import os
import subprocess
import sys

import pytest

from deepspeedsyclsupport_amd.launcher import runner as dsrun
from deepspeedsyclsupport_amd.launcher.launch import build_rank_envs, parse_core_list

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def test_parse_hostfile():
    pool = dsrun.parse_hostfile_lines(["# comment", "worker-0 slots=8", "", "worker-1 slots=4"])
    assert list(pool.items()) == [("worker-0", 8), ("worker-1", 4)]
    with pytest.raises(ValueError):
        dsrun.parse_hostfile_lines(["worker-0 slots=8", "worker-0 slots=8"])
    with pytest.raises(ValueError):
        dsrun.parse_hostfile_lines(["worker-0 8"])
    with pytest.raises(ValueError):
        dsrun.parse_hostfile_lines(["# only comments"])


def test_include_exclude():
    pool = {"w0": 4, "w1": 4}
    assert dsrun.parse_inclusion_exclusion(pool, "w0@w1:0,2", "") == {"w0": [0, 1, 2, 3], "w1": [0, 2]}
    assert dsrun.parse_inclusion_exclusion(pool, "", "w1:0") == {"w0": [0, 1, 2, 3], "w1": [1, 2, 3]}
    assert dsrun.parse_inclusion_exclusion(pool, "", "w0") == {"w1": [0, 1, 2, 3]}
    assert list(dsrun.parse_inclusion_exclusion(pool, "w1@w0", "")) == ["w0", "w1"]  # hostfile order kept
    with pytest.raises(ValueError):
        dsrun.parse_inclusion_exclusion(pool, "w0", "w1")
    with pytest.raises(ValueError):
        dsrun.parse_inclusion_exclusion(pool, "w9", "")
    with pytest.raises(ValueError):
        dsrun.parse_inclusion_exclusion(pool, "w0:7", "")


def test_world_info_and_rank_envs():
    wi = {"a": [0, 1], "b": [2, 3, 5]}
    assert dsrun.decode_world_info(dsrun.encode_world_info(wi)) == wi
    envs = build_rank_envs(wi, 1, "10.0.0.1", 1234)
    assert [e["RANK"] for e in envs] == ["2", "3", "4"]
    assert all(e["WORLD_SIZE"] == "5" and e["LOCAL_SIZE"] == "3" and e["CROSS_RANK"] == "1" for e in envs)
    assert envs[0]["HIP_VISIBLE_DEVICES"] == "2,3,5" and envs[0]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert parse_core_list("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]


def test_runner_cmds():
    args = dsrun.parse_args(["--launcher", "openmpi", "--master_addr", "w0", "train.py", "--x", "1"])
    from deepspeedsyclsupport_amd.launcher.multinode_runner import OpenMPIRunner, PDSHRunner, SlurmRunner
    active = {"w0": [0, 1], "w1": [0, 1]}
    r = OpenMPIRunner(args, "WI", active)
    r.add_export("RCCL_DEBUG", "INFO")
    cmd = r.get_cmd({}, active)
    assert cmd[:3] == ["mpirun", "-n", "4"] and "RCCL_DEBUG=INFO" in cmd and cmd[-3:] == ["train.py", "--x", "1"]
    cmd = PDSHRunner(args, "WI", active).get_cmd({}, active)
    assert "w0,w1" in cmd and "--world_info=WI" in cmd
    cmd = SlurmRunner(args, "WI", active).get_cmd({}, active)
    assert cmd[:3] == ["srun", "-n", "4"]


def test_local_launch_two_ranks(tmp_path):
    script = tmp_path / "train.py"
    script.write_text(
        "import os, sys\n"
        "import argparse\n"
        "p = argparse.ArgumentParser(); p.add_argument('--local_rank', type=int); p.add_argument('--out')\n"
        "a = p.parse_args()\n"
        "open(os.path.join(a.out, 'r' + os.environ['RANK']), 'w').write(\n"
        "    ','.join([os.environ['LOCAL_RANK'], os.environ['WORLD_SIZE'], str(a.local_rank)]))\n")
    env = dict(os.environ, PYTHONPATH=REPO)
    subprocess.run([sys.executable, "-m", "deepspeedsyclsupport_amd.launcher.runner", "--num_gpus", "2",
                    "--master_port", "29611", str(script), "--out", str(tmp_path)], check=True, env=env, cwd=REPO,
                   timeout=120)
    assert (tmp_path / "r0").read_text() == "0,2,0"
    assert (tmp_path / "r1").read_text() == "1,2,1"


def test_failed_rank_fails_launch(tmp_path):
    script = tmp_path / "bad.py"
    script.write_text("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(60)\n")
    env = dict(os.environ, PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-m", "deepspeedsyclsupport_amd.launcher.runner", "--num_gpus", "2",
                        "--no_local_rank", str(script)], env=env, cwd=REPO, timeout=60)
    assert r.returncode == 3
