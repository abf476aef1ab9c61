"""run.log layout vs the reference's own readers (CPU).

analysis/load_data.m:18-22 and symplectic_full_fourier.m:72-76 read the
parameter block with textscan at fixed header offsets (10, then 7).  The
emulator in matlab_textscan.py follows textscan's HeaderLines semantics; it is
pinned here on the head of a reference job log
(tests/golden/runlog_ref_head.txt = analysis/job-37011720/run-16/run.log
lines 1-30 + its last 3 lines), then run on the files this library writes.
The drivers' own run.log files are parsed in tests/test_gpu_qg.py."""
import os

import numpy as np
import pytest

from swraytracing_amd.runlog import PREAMBLE_LINES, RunLog, parameter_block, preamble
from tests.matlab_textscan import Fid, load_data_header

HERE = os.path.dirname(__file__)


def test_textscan_emulator_on_reference_log():
    h = load_data_header(os.path.join(HERE, "golden", "runlog_ref_head.txt"))
    assert h["resolution"] == (256, 256)
    assert h["Npackets"] == 50
    assert h["f"] == 3.0 and h["Cg"] == 1.0
    assert h["Ug"] == (0.2, 0.202628)


def test_textscan_headerlines_counts_rest_of_current_line():
    fid = Fid("a 1\nb 2\nc 3\nd 4\n")
    assert fid.textscan("a %d", 1) == [[1]]
    # the rest of line 1 is the first header line: 2 header lines -> line 3
    assert fid.textscan("c %d", 1, headerlines=2) == [[3]]


def test_header_at_line_one_does_not_parse():
    """The round-2 layout (parameter block on line 1) loses Npackets."""
    txt = parameter_block(64, 500, 12.0, 0.01, 10.0, 1.0, 10, 25, 3.0, 1.0, 0.2, 0.21, 0.21, 3.0)
    fid = Fid(txt)
    assert fid.textscan("Resolution: %dx%d", 1, headerlines=10) == [[], []]


@pytest.mark.parametrize("two_layer", [False, True])
def test_runlog_parses_with_load_data(tmp_path, two_layer):
    p = tmp_path / "run.log"
    log = RunLog(str(p))
    log(parameter_block(512, 1000000, 12.0, 0.0123, 2000.0, 333.3, 10, 25, 3.0, 1.0, 0.2, 0.2031, 0.2031, 3.0,
                        two_layer=two_layer))
    log.start()
    for s in range(1, 200):
        if two_layer and s == 120:
            log("CFL condition not met, max|u|=0.300000, new dt=0.010000\n")
        log.progress(s, 199)
    log.finish()
    log.close()
    lines = open(p).read().split("\n")
    assert lines[PREAMBLE_LINES].startswith("Resolution: 512x512")
    assert lines[-2].startswith("Real time elapsed: ") and lines[-2].endswith(" seconds")
    assert "Simulation progress:  0.00% 25.63%\n 51.26%\n" in open(p).read()  # MATLAB "% 6.2f%%"
    h = load_data_header(str(p))
    assert h == dict(resolution=(512, 512), Npackets=1000000, f=3.0, Cg=1.0, Ug=(0.2, 0.2031))


def test_preamble_is_ten_lines():
    assert preamble().count("\n") == PREAMBLE_LINES
    assert np.all([len(x) < 120 for x in preamble().split("\n")])
