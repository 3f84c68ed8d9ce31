"""CPU tests of the genotype writers (guacamole_amd/output.py)."""
from guacamole_amd.output import germline_genotype, somatic_genotype, write_json, write_vcf


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


def test_json_lines(tmp_path):
    p = tmp_path / "x.json"
    write_json(str(p), [germline_genotype("1", 5, "default", ("Alt", "Alt"), "C", "G")])
    assert '"alternateAllele": "G"' in open(p).read()
