"""bench.py's launch contract: `--gpus N` is honoured in both launch forms, never silently
replaced by the one-GPU headline (the driver's SCALE runs read n_gpus and the workload)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    return env


def test_gpus_without_devices_fails_loudly():
    """--gpus 2 in one process with fewer than 2 devices exits non-zero with a message."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two devices are present")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                         capture_output=True, text=True, env=_env(), timeout=300)
    assert out.returncode != 0
    assert "needs 2 GPUs" in out.stderr
    assert out.stdout.strip() == ""


def test_gpus_mismatch_with_world_size_fails():
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode != 0 and "WORLD_SIZE=4" in out.stderr


@pytest.mark.gpu
def test_bench_group_one_device(capsys):
    """`bench.py --gpus 4 --one-device`: the library's multi-GPU engine (4 shards on one GPU,
    the same code path as 4 devices) with the same-job one-GPU base of the same window."""
    sys.path.insert(0, ROOT)
    import bench

    out = bench.main(["--gpus", "4", "--one-device", "--workload", "custom", "--n", "1000000",
                      "--window", "20", "--steps", "2", "--warmup", "1"])
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line == json.loads(json.dumps(out))
    assert line["n_gpus"] == 4 and line["devices"] == 1 and line["scaling"] == "strong"
    assert line["config"]["workload"] == "1000000 Imp3D push-sum, 20-round window"
    assert line["config"]["rounds_per_step"] == 20
    pr = line["per_rank"]
    assert pr["world"] == 4 and 0 < pr["actors"] < line["config"]["actors"]
    assert pr["round_kernel_ms_device_shared"] > 0 and "round_kernel_ms" not in pr  # one device: not per rank
    base = line["strong_scaling_base"]
    assert base["rounds_per_step"] == 20 and base["value"] > 0
    assert base["t1_over_n_tn"] == pytest.approx(line["value"] / (4 * base["value"]))
    assert line["roofline"]["launches"] > 0
