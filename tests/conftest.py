import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def _ensure_built():
    import __graft_entry__

    __graft_entry__.build()


_ensure_built()


@pytest.fixture(scope="session")
def small_model():
    """Small 3D model (10^3 grid, 3 elements x 4 ions, ~3k lines): seconds on the CPU oracle."""
    from artis_amd.model import Model

    m = Model(ngrid_1d=10, nlevels_per_ion=60, n_ionising=20, max_lines=8000, ntstep=30)
    return m


@pytest.fixture(scope="session")
def shell_model():
    """1D 12-shell model mapped onto a 12^3 cuboid (map_1dmodeltogrid, grid.cc:910-940)."""
    from artis_amd.model import Model

    return Model(ngrid_1d=12, nshells_1d=12, nlevels_per_ion=40, n_ionising=15, max_lines=4000, ntstep=30)
