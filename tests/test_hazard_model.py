"""CPU test of the packet-buffer hazard checker's model (swrt_hazard.hpp):
tests/hazard_model.cpp replays the multi-stream launch protocol of
swrt_api.hip abstractly and checks the checker's verdicts — silent on the
library's ordering (third buffers, joins before re-binnings and whole
launches), reporting the pre-third-buffer race, a whole launch or a
re-binning without a join, and round 4's skewed cycle-end share (its regions
are the band slots swrt_share.hpp's mapping gives each part).  The device-side counterpart is
tests/test_gpu_hazard.py."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hazard_checker_model(tmp_path):
    exe = tmp_path / "hazard_model"
    # hipcc: the model includes swrt_share.hpp (host/device mapping functions);
    # host code only, no GPU needed
    subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "--offload-arch=gfx950", "-O1", "-std=c++17",
                    "-Wall", "-Werror", "-o", str(exe), os.path.join(ROOT, "tests", "hazard_model.cpp")], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
    assert "legacy_park_reported_s2 ok" in r.stdout
    assert "skewed_cycle_end_reported ok" in r.stdout and "consistent_skew_silent ok" in r.stdout
    assert "share_partitions_slots ok" in r.stdout
    assert "sort launch" in r.stdout or "part" in r.stdout
