"""CPU-side checks of the C-ABI library: it loads and exports every symbol gqpileup.h declares."""
import os
import re

from conftest import ROOT
from guacamole_amd import native


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "gqpileup.h")).read()
    declared = set(re.findall(r"\b(gq_[a-z_]+)\s*\(", hdr))
    L = native.lib()
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert set(native.EXPORTED) == declared
    assert b"gfx950" in L.gq_version()


def test_ingest_library_exports_every_declared_symbol():
    from guacamole_amd import ingest
    from guacamole_amd.build import build_ingest
    build_ingest()
    hdr = open(os.path.join(ROOT, "include", "gqingest.h")).read()
    declared = set(re.findall(r"\b(gq_[a-z0-9_]+)\s*\(", hdr))
    assert {"gq_bam_open", "gq_bam_scan", "gq_bam_fill", "gq_md_count", "gq_md_fill"} <= declared
    L = ingest.lib()
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing


def test_bam_map_on_the_host(tmp_path):
    """gq_bam_dev_map (the host half of the device BAM load: file map + BGZF block table) needs
    no GPU: BAM -> mapped, plain gzip -> not BGZF (the host loader's case), errors as ReadLoadError."""
    import gzip
    import pytest
    from guacamole_amd import bamdev
    from guacamole_amd.reads import ReadLoadError
    from conftest import fixture
    m = bamdev.MappedBam(fixture("chrM.sorted.bam"))
    assert m.ok and m.h
    m.close()
    g = tmp_path / "plain.gz"
    with gzip.open(g, "wb") as fh:
        fh.write(b"BAM\1" + b"\0" * 100)
    assert not bamdev.MappedBam(str(g)).ok
    with pytest.raises(ReadLoadError):
        bamdev.MappedBam(str(tmp_path / "missing.bam"))
    bad = tmp_path / "bad.bam"
    bad.write_bytes(b"not a bam at all" * 10)
    with pytest.raises(ReadLoadError):
        bamdev.MappedBam(str(bad))
    joined = bamdev.map_bams([fixture("chrM.sorted.bam")])["join"]()
    assert joined[fixture("chrM.sorted.bam")].ok
