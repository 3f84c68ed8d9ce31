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


def test_somatic_rows_from_columns():
    """SomaticCalls.rows builds its dicts from column lists (one tolist per column): the same rows,
    field for field and type for type, as indexing the numpy columns element by element."""
    import numpy as np
    from guacamole_amd import native as N
    n = 257
    rng = np.random.default_rng(7)
    cols = {k: rng.integers(0, 9, n).astype(dt) for k, dt in
            (("contig", np.int32), ("pos", np.int32), ("sample", np.int32), ("ref_len", np.int32),
             ("alt_len", np.int32), ("gq", np.int32), ("flags", np.int32))}
    cols["ref_off"] = rng.integers(0, 100, n).astype(np.int64)
    cols["alt_off"] = rng.integers(0, 100, n).astype(np.int64)
    cols["log_odds"] = rng.random(n) * 50
    for s in ("tumor", "normal"):
        a = np.zeros(n, dtype=N._EVIDENCE_DTYPE)
        for f in N.EVIDENCE_FIELDS:
            a[f] = rng.random(n) * 100
        cols[s] = a
    pool = bytes(rng.integers(65, 91, 120).astype(np.uint8))
    got = N.SomaticCalls(cols, pool, 0, 0).rows
    c = cols
    ev = lambda e: tuple(e[k].item() for k in N.EVIDENCE_FIELDS)  # noqa: E731
    want = [dict(contig=int(c["contig"][i]), locus=int(c["pos"][i]), sample=int(c["sample"][i]),
                 ref=pool[c["ref_off"][i]:c["ref_off"][i] + c["ref_len"][i]].decode("latin-1"),
                 alt=pool[c["alt_off"][i]:c["alt_off"][i] + c["alt_len"][i]].decode("latin-1"),
                 log_odds=float(c["log_odds"][i]), gq=int(c["gq"][i]), tumor=ev(c["tumor"][i]),
                 normal=ev(c["normal"][i]), flags=int(c["flags"][i])) for i in range(n)]
    assert got == want
    assert all(type(a) is type(b) for r, w in zip(got, want) for a, b in zip(r.values(), w.values()))
    assert N.SomaticCalls({k: v[:0] for k, v in cols.items()}, b"", 0, 0).rows == []
