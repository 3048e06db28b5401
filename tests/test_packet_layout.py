"""Host check of the packet store layout (artis_amd/csrc/engine/packet_soa.h): tests/packet_layout_check.cpp, built
with hipcc for the host (no GPU needed) -- distinct store words for every packet's 38 words, the line-absorption and
deactivation words in their own 64-byte sectors of the cold record, line-aligned hot records."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_packet_store_layout(tmp_path):
    exe = tmp_path / "packet_layout_check"
    subprocess.run([HIPCC, "-std=c++17", "-O1", "-I", os.path.join(REPO, "include"),
                    "-I", os.path.join(REPO, "artis_amd", "csrc", "engine"),
                    os.path.join(REPO, "tests", "packet_layout_check.cpp"), "-o", str(exe)], check=True,
                   capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad 0" in r.stdout
