"""bench.py reports roofline.traffic from a committed PMC summary only when
that summary was collected on the library being timed: the same libacm.so
bytes, or a rebuild of the very same sources (hipcc output is not
byte-reproducible).  Anything else is reported as null with the reason
(stale counters must not be attributed to a new build)."""
import json
import os
import shutil

import pytest

import bench
from apex_camera_models import _lib

WL = "kb_project_jacobian_f64_aos"


def _write(tmp_path, **fields):
    prof = tmp_path / "profiles"
    prof.mkdir(exist_ok=True)
    d = {"workload": WL, "points": 10_000_000, "hbm_bytes_per_launch": 1.7e9}
    d.update(fields)
    (prof / "x_pmc_test.json").write_text(json.dumps(d))


@pytest.fixture
def root(tmp_path, monkeypatch):
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libacm.so not built")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    # sources for the mtime check: copy the real ones (older than the library)
    src = os.path.dirname(os.path.dirname(_lib.LIB_PATH))
    shutil.copytree(os.path.join(src, "csrc"), tmp_path / "apex-camera-models_amd" / "csrc")
    (tmp_path / "include").mkdir()
    shutil.copy(os.path.join(os.path.dirname(src), "include", "acm.h"), tmp_path / "include")
    for f in (tmp_path / "apex-camera-models_amd" / "csrc").iterdir():
        os.utime(f, (0, 0))
    os.utime(tmp_path / "include" / "acm.h", (0, 0))
    return tmp_path


def test_same_library_bytes(root):
    _write(root, libacm_sha256=bench.lib_sha256())
    t, src = bench.load_traffic(WL, 10_000_000)
    assert t == 1.7e9 and src.endswith("x_pmc_test.json")


def _ident():
    from apex_camera_models import _buildinfo
    return _buildinfo.lib_identity(_lib.LIB_PATH)


def test_rebuild_of_same_sources(root):
    _write(root, libacm_sha256="0" * 64, libacm_source_sha256=_lib.source_sha256(),
           libacm_identity=_ident())
    t, src = bench.load_traffic(WL, 10_000_000)
    assert t == 1.7e9 and "same libacm sources" in src


def test_same_sources_other_build_variant_is_not_reported(root):
    """a summary collected on a diagnostic / A-B build of the same
    sources (another file, other -D defines in acm_version) is not this
    library's traffic; neither is one that does not name its build."""
    for ident in ({"name": "libacm_diag1.so", "version": _ident()["version"]},
                  {"name": "libacm.so", "version": "acm 0.3.0 (gfx950; ACM_DIAG_SAMPLE)"},
                  None):
        _write(root, libacm_sha256="0" * 64, libacm_source_sha256=_lib.source_sha256(),
               libacm_identity=ident)
        t, src = bench.load_traffic(WL, 10_000_000)
        assert t is None and "stale" in src, ident


def test_other_build_is_not_reported(root):
    _write(root, libacm_sha256="0" * 64, libacm_source_sha256="1" * 64)
    t, src = bench.load_traffic(WL, 10_000_000)
    assert t is None and "stale" in src


def test_sources_newer_than_library_are_not_trusted(root):
    _write(root, libacm_sha256="0" * 64, libacm_source_sha256=_lib.source_sha256(),
           libacm_identity=_ident())
    f = root / "apex-camera-models_amd" / "csrc" / "acm.hip"
    future = os.path.getmtime(_lib.LIB_PATH) + 100
    os.utime(f, (future, future))
    t, src = bench.load_traffic(WL, 10_000_000)
    assert t is None


def test_other_workload_or_size(root):
    _write(root, libacm_sha256=bench.lib_sha256())
    assert bench.load_traffic(WL, 1_000_000)[0] is None
    assert bench.load_traffic("kb_project_f64_aos", 10_000_000)[0] is None


def test_matching_summary_wins_over_a_later_named_stale_one(root):
    """Several summaries of the workload: the one collected on this library
    is reported even when a stale one sorts after it by file name."""
    prof = root / "profiles"
    prof.mkdir(exist_ok=True)
    base = {"workload": WL, "points": 10_000_000}
    (prof / "a_pmc_match.json").write_text(json.dumps(
        {**base, "hbm_bytes_per_launch": 1.7e9, "libacm_sha256": bench.lib_sha256()}))
    (prof / "z_pmc_stale.json").write_text(json.dumps(
        {**base, "hbm_bytes_per_launch": 9.9e9, "libacm_sha256": "0" * 64,
         "libacm_source_sha256": "1" * 64}))
    t, src = bench.load_traffic(WL, 10_000_000)
    assert t == 1.7e9 and src.endswith("a_pmc_match.json")
