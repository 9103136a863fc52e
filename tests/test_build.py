"""Build provenance (no GPU): the in-tree library carries the digest of the
sources it was built from, and a library that does not match them is refused."""
import pytest

from jwave_amd import _build, _lib
from jwave_amd.exceptions import JWaveError


def test_stamp_matches_sources():
    _lib.lib()
    p = _lib.provenance()
    assert p["matches_sources"], p
    assert len(p["lib_sha256"]) == 16 and p["hipcc"]


def test_stale_library_refused(monkeypatch):
    monkeypatch.setattr(_build, "source_digest", lambda: "0" * 64)
    assert _build.stale()
    monkeypatch.setenv("JWAVE_AMD_NO_BUILD", "1")
    monkeypatch.delenv("JWAVE_AMD_LIB", raising=False)
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(JWaveError, match="not built from these sources"):
        _lib.lib()


def test_library_reads_no_variant_switches():
    """The product library reads no environment switch that selects a kernel
    variant: its only JWV_* environment names are the
    launch log (a stderr trace, no effect on results)."""
    import re
    from jwave_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    names = set(re.findall(rb"JWV_[A-Z0-9_]+", blob))
    allowed = {b"JWV_LAUNCH", b"JWV_LAUNCH_LOG", b"JWV_TRANSFORM_FWT", b"JWV_TRANSFORM_WPT"}
    assert names <= allowed, sorted(names - allowed)
    assert b"JWV_WPT_DIAGW" not in blob
