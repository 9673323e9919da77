"""The oracle's status decisions on points placed on every threshold of the
hot path (tests/boundary_probes.py: +-8 ulps around each root) equal an
independent binary64 emulation of the reference's Rust conditions (mpmath,
53-bit round-to-nearest).  tests/test_gpu_parity.py holds the HIP kernels to
the oracle on the same probes."""
import numpy as np
import pytest

import boundary_probes as B
import oracle as O

FAMILIES = B.probes()


@pytest.mark.parametrize("fam", range(len(FAMILIES)),
                         ids=lambda i: f"m{FAMILIES[i][0]}_{FAMILIES[i][3]}_{i}")
def test_oracle_status_on_thresholds(fam):
    model, p, (w, h), kind, pts = FAMILIES[fam]
    if kind == "project":
        _, st, _ = O.project(model, p, w, h, pts)
    else:
        _, st = O.unproject(model, p, w, h, pts)
    emu = np.array([B.emulate_status(model, p, w, h, kind, q) for q in pts])
    bad = np.nonzero(st != emu)[0]
    assert bad.size == 0, [(pts[i].tolist(), int(st[i]), int(emu[i])) for i in bad[:5]]


def test_probes_straddle_their_thresholds():
    """every family exercises both outcomes of at least one of its decisions"""
    for model, p, (w, h), kind, pts in FAMILIES:
        emu = {B.emulate_status(model, p, w, h, kind, q) for q in pts}
        assert len(emu) > 1, (model, kind, emu)
