"""Launcher / elasticity / env report (reference tests/unit/launcher/test_run.py, test_multinode_runner.py,
tests/unit/elasticity/test_elastic.py strategies: pure argument/resource parsing, command construction, and
one real single-node launch of a tiny script)."""
import os
import subprocess
import sys

import pytest

from hcache_deepspeed_amd.launcher import runner as R


def test_hostfile_parsing_and_errors():
    pool = R._parse_hostfile(["worker-0 slots=8", "# comment", "", "worker-1 slots=4  "])
    assert list(pool.items()) == [("worker-0", 8), ("worker-1", 4)]
    with pytest.raises(ValueError):
        R._parse_hostfile(["worker-0 slots=8", "worker-0 slots=8"])
    with pytest.raises(ValueError):
        R._parse_hostfile(["worker-0 8"])
    with pytest.raises(ValueError):
        R._parse_hostfile(["# only comments"])


def test_include_exclude_filters():
    pool = {"worker-0": 4, "worker-1": 4}
    a = R.parse_inclusion_exclusion(pool, "worker-0@worker-1:0,2", "")
    assert dict(a) == {"worker-0": [0, 1, 2, 3], "worker-1": [0, 2]}
    b = R.parse_inclusion_exclusion(pool, "", "worker-1:0")
    assert dict(b) == {"worker-0": [0, 1, 2, 3], "worker-1": [1, 2, 3]}
    c = R.parse_inclusion_exclusion(pool, "", "worker-0")
    assert dict(c) == {"worker-1": [0, 1, 2, 3]}
    with pytest.raises(ValueError):
        R.parse_inclusion_exclusion(pool, "worker-0", "worker-1")
    with pytest.raises(ValueError):
        R.parse_inclusion_exclusion(pool, "worker-2", "")
    with pytest.raises(ValueError):
        R.parse_inclusion_exclusion(pool, "worker-0:7", "")


def test_world_info_roundtrip_and_num_nodes():
    wi = {"a": [0, 1], "b": [3]}
    assert R.decode_world_info(R.encode_world_info(wi)) == wi
    assert R.parse_num_nodes("2", False) == (2, -1)
    assert R.parse_num_nodes("1:4", True) == (1, 4)
    with pytest.raises(RuntimeError):
        R.parse_num_nodes("1:4", False)


def test_launch_env_and_rank_mapping():
    from hcache_deepspeed_amd.launcher import launch as L
    wi = {"a": [0, 1, 2, 3], "b": [0, 1]}
    env, ranks = L.build_env({}, wi, 1, "10.0.0.1", 1234)
    assert ranks == [4, 5] and env["WORLD_SIZE"] == "6" and env["LOCAL_SIZE"] == "2"
    assert env["CROSS_RANK"] == "1" and env["CROSS_SIZE"] == "2" and env["HIP_VISIBLE_DEVICES"] == "0,1"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_multinode_runner_commands():
    from hcache_deepspeed_amd.launcher.multinode_runner import RUNNERS
    args = R.parse_args(["--launcher", "pdsh", "--master_addr", "w0", "train.py", "--lr", "1"])
    active = {"w0": [0, 1], "w1": [0, 1]}
    cmd = RUNNERS["pdsh"](args, "XYZ", active).get_cmd({}, active)
    assert cmd[:6] == ["pdsh", "-S", "-f", "1024", "-w", "w0,w1"]
    assert "--node_rank=%n" in cmd and "--world_info=XYZ" in cmd and cmd[-3:] == ["train.py", "--lr", "1"]
    args = R.parse_args(["--launcher", "openmpi", "-H", "/tmp/hf", "train.py"])
    cmd = RUNNERS["openmpi"](args, "XYZ", active).get_cmd({}, active)
    assert cmd[:3] == ["mpirun", "-n", "4"] and "HSA_ENABLE_IPC_MODE_LEGACY=0" in cmd
    cmd = RUNNERS["slurm"](R.parse_args(["--launcher", "slurm", "train.py"]), "X", active).get_cmd({}, active)
    assert cmd[:3] == ["srun", "-n", "4"]
    cmd = RUNNERS["mpich"](R.parse_args(["--launcher", "mpich", "train.py"]), "X", active).get_cmd({}, active)
    assert cmd[:5] == ["mpirun", "-n", "4", "-ppn", "2"]


def test_single_node_launch_end_to_end(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(
        "import os, sys\n"
        "lr = [a for a in sys.argv if a.startswith('--local_rank=')][0].split('=')[1]\n"
        "assert lr == os.environ['LOCAL_RANK']\n"
        "open(os.path.join(sys.argv[-1], 'rank' + os.environ['RANK']), 'w').write(os.environ['WORLD_SIZE'])\n")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    rc = subprocess.call([sys.executable, "-m", "hcache_deepspeed_amd.launcher.runner", "--num_gpus", "3",
                          "--hostfile", str(tmp_path / "none"), str(script), str(tmp_path)], env=env, timeout=120)
    assert rc == 0
    assert sorted(os.listdir(tmp_path)) == ["child.py", "rank0", "rank1", "rank2"]
    assert (tmp_path / "rank2").read_text() == "3"


def test_launch_propagates_failure(tmp_path):
    script = tmp_path / "bad.py"
    script.write_text("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(60)\n")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    rc = subprocess.call([sys.executable, "-m", "hcache_deepspeed_amd.launcher.runner", "--num_gpus", "2",
                          "--hostfile", str(tmp_path / "none"), str(script)], env=env, timeout=60)
    assert rc == 3


def test_elastic_config_v01_v02():
    from hcache_deepspeed_amd.elasticity import compute_elastic_config, ElasticityIncompatibleWorldSize
    cfg = {"elasticity": {"enabled": True, "max_train_batch_size": 10000, "micro_batch_sizes": [8, 12, 16, 17],
                          "min_gpus": 32, "max_gpus": 1500, "min_time": 20, "version": 0.1}}
    bs, gpus = compute_elastic_config(cfg, "0.16.8")
    assert bs == 9792 and len(gpus) == 23 and gpus[0] == 32 and gpus[-1] == 1224
    bs2, gpus2, mbs = compute_elastic_config(cfg, "0.16.8", world_size=64)
    assert bs2 == bs and mbs == 17 and 64 in gpus2
    with pytest.raises(ElasticityIncompatibleWorldSize):
        compute_elastic_config(cfg, "0.16.8", world_size=33)
    cfg2 = {"elasticity": {"enabled": True, "max_train_batch_size": 2000, "micro_batch_sizes": [2, 4, 6],
                           "min_gpus": 1, "max_gpus": 10000, "num_gpus_per_node": 8, "version": 0.2}}
    bs, gpus, mbs = compute_elastic_config(cfg2, "0.16.8", world_size=16, return_microbatch=True)
    assert bs % (16 * mbs) == 0 and 16 in gpus


def test_env_report_runs(capsys):
    from hcache_deepspeed_amd.env_report import cli_main
    cli_main([])
    out = capsys.readouterr().out
    assert "fused_adam" in out and "torch version" in out
