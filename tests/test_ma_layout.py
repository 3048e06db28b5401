"""Host check of the macro-atom key-record layout (engine_dev.h ma_layout / ma_rec_pos) and of the two-line search
k_ma makes over it: tests/ma_layout_check.cpp, built with hipcc for the host (no GPU needed), run over every
(down, up) array-size shape up to 300 x 700.  Covers the round-5 line-0 suffix and the round-4 separators-only
layout (-DARTIS_MA_SUFFIX=0)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("suffix", [1, 0])
def test_ma_record_layout_and_search(tmp_path, suffix):
    exe = tmp_path / "ma_layout_check"
    subprocess.run([HIPCC, "-std=c++17", "-O1", f"-DARTIS_MA_SUFFIX={suffix}", "-I", os.path.join(REPO, "include"),
                    "-I", os.path.join(REPO, "artis_amd", "csrc", "engine"),
                    os.path.join(REPO, "tests", "ma_layout_check.cpp"), "-o", str(exe)], check=True,
                   capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad 0" in r.stdout
