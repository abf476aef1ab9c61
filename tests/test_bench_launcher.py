"""bench.py's launcher logic (CPU): `--gpus N` without a torch.distributed
environment runs the ranks as a child torch.distributed.run; inside one,
WORLD_SIZE must agree with --gpus.  Importing bench does not import torch."""
import sys

import pytest

import bench


def test_import_is_light():
    assert "torch" not in vars(bench) or vars(bench)["torch"] is None


def test_one_gpu_runs_in_process():
    a = bench.parse_args([])
    assert bench.launcher_cmd(a, [], {}) is None
    a = bench.parse_args(["--gpus", "1"])
    assert bench.launcher_cmd(a, ["--gpus", "1"], {}) is None


def test_n_gpus_launches_child_torchrun():
    argv = ["--gpus", "4", "--steps", "7"]
    cmd = bench.launcher_cmd(bench.parse_args(argv), argv, {})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-3:] == ["--gpus", "4", "--steps", "7"][-3:] and cmd[-4] == "--gpus"
    assert cmd[cmd.index("--master-addr=127.0.0.1") + 2].endswith("bench.py")


def test_rank_checks_world_size():
    a = bench.parse_args(["--gpus", "8"])
    assert bench.launcher_cmd(a, [], {"WORLD_SIZE": "8"}) is None
    with pytest.raises(SystemExit):
        bench.launcher_cmd(a, [], {"WORLD_SIZE": "2"})
    # no --gpus under torch.distributed.run: WORLD_SIZE decides
    assert bench.launcher_cmd(bench.parse_args([]), [], {"WORLD_SIZE": "2"}) is None


def test_strong_scaling_is_default():
    a = bench.parse_args([])
    assert a.scaling == "strong" and a.packets == 1_000_000
    assert bench.parse_args(["--scaling", "weak"]).scaling == "weak"


def test_relay_forwards_only_the_metric_line(capfd):
    code = ("import json,sys;print('noise');print(json.dumps({'metric':'m','value':1}));"
            "print('more', file=sys.stderr);sys.exit(3)")
    rc = bench.relay([sys.executable, "-c", code])
    out, err = capfd.readouterr()
    assert rc == 3
    assert out.strip() == '{"metric": "m", "value": 1}'
    assert "noise" in err and "more" in err


@pytest.mark.parametrize("world", [1, 2, 8])
def test_shards_cover_the_ensemble(world):
    from swraytracing_amd.dist import shard_range
    n = 1_000_000
    r = [shard_range(n, world, i) for i in range(world)]
    assert r[0][0] == 0 and r[-1][1] == n
    assert all(r[i][1] == r[i + 1][0] for i in range(world - 1))
    assert r[0][1] - r[0][0] == -(-n // world)
