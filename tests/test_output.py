"""CPU tests of the genotype writers (guacamole_amd/output.py)."""
import json

import pytest

from guacamole_amd.output import (GENOTYPE_SCHEMA, VARIANT_SCHEMA, dbsnp_join, germline_genotype, java_float,
                                  read_avro_json, read_dbsnp_vcf, somatic_genotype, write_json, write_vcf)


def test_vcf_lines(tmp_path):
    g = [germline_genotype("chrM", 72, "s1", ("Ref", "Alt"), "T", "C"),
         germline_genotype("chrM", 300, "s1", ("Alt", "Alt"), "A", "AC")]
    row = dict(locus=99, ref="G", alt="A", gq=42, tumor=(0.9, 50, 10, 20, 5, 60.0, 60.0, 30.0, 30.0, 1.0))
    g.append(somatic_genotype("chrM", row, "s1"))
    p = tmp_path / "x.vcf"
    write_vcf(str(p), g, {"chrM": 16571})
    body = [l.rstrip("\n").split("\t") for l in open(p) if not l.startswith("#")]
    assert body[0][:5] == ["chrM", "73", ".", "T", "C"] and body[0][-1] == "0/1"
    assert body[1][-1] == "1/1"
    assert body[2][8] == "GT:GQ:DP:AD" and body[2][-1] == "0/1:42:50:40,10"
    assert g[2]["expectedAlleleDosage"] == 0.20000000298023224  # float32(10) / float32(50)


def _records(text):
    return read_avro_json(text)


def test_json_avro_field_sets(tmp_path):
    """The JSON writer emits what Avro's JsonEncoder writes for the bdg-formats Genotype schema:
    every field in schema order, unions wrapped; the germline builder sets no `end` and no depths
    (GermlineThresholdCaller.scala:106-117), the somatic one its AlleleConversions fields
    (AlleleConversions.scala:47-62) with end = start + 1 (CalledSomaticAllele.scala:46)."""
    p = tmp_path / "x.json"
    row = dict(locus=99, ref="G", alt="A", gq=42, tumor=(0.9, 50, 10, 20, 5, 60.0, 60.0, 30.0, 30.0, 1.0))
    write_json(str(p), [germline_genotype("1", 5, "default", ("Alt", "Alt"), "C", "G"),
                        somatic_genotype("chrM", row, "s1")])
    text = open(p).read()
    assert text.endswith("}\n") and '"alleles" : [ "Alt", "Alt" ]' in text
    g, s = _records(text)
    assert list(g) == [f for f, _, _ in GENOTYPE_SCHEMA] == list(s)
    gv = g["variant"]["org.bdgenomics.formats.avro.Variant"]
    assert list(gv) == [f for f, _, _ in VARIANT_SCHEMA]
    assert gv["end"] is None and gv["start"] == {"long": 5}
    assert gv["contig"]["org.bdgenomics.formats.avro.Contig"]["contigName"] == {"string": "1"}
    assert gv["referenceAllele"] == {"string": "C"} and gv["alternateAllele"] == {"string": "G"}
    assert g["readDepth"] is None and g["genotypeQuality"] is None and g["sampleId"] == {"string": "default"}
    sv = s["variant"]["org.bdgenomics.formats.avro.Variant"]
    assert sv["start"] == {"long": 99} and sv["end"] == {"long": 100}
    assert s["alleles"] == ["Ref", "Alt"] and s["genotypeQuality"] == {"int": 42}
    assert s["readDepth"] == {"int": 50} and s["referenceReadDepth"] == {"int": 40}
    assert s["alternateReadDepth"] == {"int": 10} and s["expectedAlleleDosage"] == {"float": 0.2}
    assert '"float" : 0.2\n' in text


def test_java_float_rendering():
    assert [java_float(x) for x in (0.2, 1e-4, 1.0, 12345678.0, 1 / 3, 0.001)] == [
        "0.2", "1.0E-4", "1.0", "1.2345678E7", "0.33333334", "0.001"]


def test_max_genotypes_and_dbsnp(tmp_path):
    from guacamole_amd.commands import _write_genotypes
    g = [germline_genotype("1", 5, "default", ("Alt", "Alt"), "C", "G")]
    _write_genotypes(str(tmp_path / "a.json"), g, max_genotypes=1)  # fraction 1.0: everything
    assert len(_records(open(tmp_path / "a.json").read())) == 1
    with pytest.raises(ValueError, match="must be on interval"):
        _write_genotypes(str(tmp_path / "b.json"), g, max_genotypes=5)
    vcf = tmp_path / "dbsnp.vcf"
    vcf.write_text("##fileformat=VCFv4.1\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n"
                   "20\t100\trs42\tG\tA,T\t.\t.\t.\n20\t100\trs43\tG\tA\t.\t.\t.\n20\t7\t.\tC\tG\t.\t.\t.\n")
    db = read_dbsnp_vcf(str(vcf))
    rows = [dict(contig="20", locus=99, ref="G", alt="A"), dict(contig="20", locus=99, ref="G", alt="C"),
            dict(contig="20", locus=6, ref="C", alt="G")]
    out = dbsnp_join(rows, db)
    assert [(r["alt"], r["rs_id"]) for r in out] == [("A", 42), ("A", 43), ("C", None), ("G", None)]
