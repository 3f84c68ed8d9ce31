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
