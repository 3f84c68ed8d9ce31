"""CPU tests of the genotype writers (guacamole_amd/output.py)."""
import json

import numpy as np
import pytest

from guacamole_amd.output import (GENOTYPE_SCHEMA, VARIANT_SCHEMA, dbsnp_join, germline_genotype, java_float,
                                  read_avro_json, read_dbsnp_vcf, somatic_genotype, write_json, write_vcf,
                                  write_vcf_dir, write_vcf_dir_germline)


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


def test_germline_vcf_writer_equals_record_writer(tmp_path):
    """write_vcf_dir_germline (the CLI's germline path, rows straight from the call columns)
    writes the bytes write_vcf_dir writes for the same germline_genotype records: one and
    three samples, every allele pair, indels, an empty call list."""
    names = ["s1", "s2", "default"]
    gts = [("Ref", "Alt"), ("Alt", "Alt"), ("Alt", "OtherAlt"), ("Ref", "Ref"), ("NoCall", "NoCall")]
    for samples in (1, 3):
        rows = [("chrM" if i % 3 else "1", 10 * i, i % samples, gts[i % len(gts)], "ACGT"[i % 4],
                 "ACGT"[(i + 1) % 4] + ("T" if i % 7 == 0 else ""), 0) for i in range(40)]
        for rs in (rows, []):
            a, b = tmp_path / ("a%d%d.vcf" % (samples, len(rs))), tmp_path / ("b%d%d.vcf" % (samples, len(rs)))
            write_vcf_dir(str(a), [germline_genotype(c, l, names[s], gt, ref, alt) for c, l, s, gt, ref, alt, _ in rs],
                          {"1": 5000, "chrM": 16571})
            write_vcf_dir_germline(str(b), rs, lambda s: names[s], {"1": 5000, "chrM": 16571})
            assert (a / "part-r-00000").read_bytes() == (b / "part-r-00000").read_bytes()
            assert (b / "_SUCCESS").exists()


def test_germline_vcf_column_writer_equals_record_writer(tmp_path):
    """write_vcf_dir_germline_calls (the CLI's single-process path: the library's line writer
    over the result columns, gq_write_vcf_germline) writes the record writer's bytes; one and
    three samples (the latter through the row layout), indels, an empty call list."""
    import numpy as np
    from guacamole_amd import native
    from guacamole_amd.output import write_vcf_dir_germline_calls
    names = ["s1", "s2", "default"]
    contigs = ["1", "chrM"]
    code = {"Ref": 0, "Alt": 1, "OtherAlt": 2, "NoCall": 3}
    gts = [("Ref", "Alt"), ("Alt", "Alt"), ("Alt", "OtherAlt"), ("Ref", "Ref"), ("NoCall", "NoCall")]
    for samples in (1, 3):
        for n in (40, 0):
            rows = [(contigs[1 if i % 3 else 0], 10 * i, i % samples, gts[i % len(gts)], "ACGT"[i % 4],
                     "ACGT"[(i + 1) % 4] + ("T" if i % 7 == 0 else ""), 0) for i in range(n)]
            pool, ro, ao = b"", [], []
            for r in rows:
                ro.append(len(pool))
                pool += r[4].encode()
                ao.append(len(pool))
                pool += r[5].encode()
            a = {"contig": np.array([contigs.index(r[0]) for r in rows], np.int32),
                 "pos": np.array([r[1] for r in rows], np.int64), "sample": np.array([r[2] for r in rows], np.uint8),
                 "gt0": np.array([code[r[3][0]] for r in rows], np.uint8),
                 "gt1": np.array([code[r[3][1]] for r in rows], np.uint8),
                 "flags": np.zeros(n, np.uint8), "ref_off": np.array(ro, np.int64),
                 "ref_len": np.array([len(r[4]) for r in rows], np.int32), "alt_off": np.array(ao, np.int64),
                 "alt_len": np.array([len(r[5]) for r in rows], np.int32)}
            calls = native.GermlineCalls(a, pool, 0, 0, 0, 0)
            x, y = tmp_path / ("x%d%d.vcf" % (samples, n)), tmp_path / ("y%d%d.vcf" % (samples, n))
            write_vcf_dir(str(x), [germline_genotype(c, l, names[s], gt, ref, alt) for c, l, s, gt, ref, alt, _ in rows],
                          {"1": 5000, "chrM": 16571})
            write_vcf_dir_germline_calls(str(y), calls, contigs, lambda s: names[s], {"1": 5000, "chrM": 16571})
            assert (x / "part-r-00000").read_bytes() == (y / "part-r-00000").read_bytes()
            assert (y / "_SUCCESS").exists()


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


def test_vcf_output_is_a_hadoop_directory(tmp_path):
    """--out X.vcf: saveAsVcf after coalesce(1) writes the directory X.vcf holding part-r-00000
    and _SUCCESS (Common.scala:290-293, README.md:49-51); an existing X.vcf is refused."""
    import os
    from guacamole_amd.commands import OutputFormatError, _write_genotypes
    g = [germline_genotype("1", 5, "default", ("Alt", "Alt"), "C", "G")]
    out = tmp_path / "calls.VCF"
    _write_genotypes(str(out), g, {"1": 100})
    assert sorted(os.listdir(out)) == ["_SUCCESS", "part-r-00000"]
    body = [l for l in open(out / "part-r-00000") if not l.startswith("#")]
    assert body == ["1\t6\t.\tC\tG\t.\t.\t.\tGT\t1/1\n"]
    with pytest.raises(OutputFormatError, match="already exists"):
        _write_genotypes(str(out), g)
    assert write_vcf_dir(str(tmp_path / "b.vcf"), g).endswith("part-r-00000")


def _plain_from_json(genotypes):
    from guacamole_amd.output import avro_json, unwrap_avro_json
    return [unwrap_avro_json("Genotype", r) for r in read_avro_json(avro_json(genotypes))]


def _same_records(a, b):
    """Field for field; float32 fields compared as float32 (the JSON text is Float.toString)."""
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x.keys() == y.keys()
        for k in x:
            if k == "expectedAlleleDosage" and x[k] is not None:
                assert np.float32(x[k]) == np.float32(y[k]) or (np.isnan(x[k]) and np.isnan(y[k])), k
            else:
                assert x[k] == y[k], k


@pytest.mark.parametrize("name", ["calls.adam", "calls.parquet", "calls", "calls.vcf.gz"])
def test_parquet_output_equals_the_avro_json_records(tmp_path, name):
    """Every other extension is ADAM Parquet (adamParquetSave, Common.scala:294-302): a Hadoop
    directory of part files whose Genotype rows, read back, equal the Avro-JSON writer's records
    field for field (byte parity with parquet-mr's files is unpinned).  An existing directory is
    refused before any work."""
    import os
    from guacamole_amd.commands import OutputFormatError, _write_genotypes, check_output_path
    from guacamole_amd.output import read_parquet_dir, somatic_genotype
    g = [germline_genotype("1", 5, "default", ("Alt", "Alt"), "C", "G"),
         germline_genotype("1", 9, "s2", ("Ref", "Alt"), "A", "AT"),
         somatic_genotype("2", dict(tumor=(0.9, 30, 7, 10, 3), gq=44, locus=99, ref="A", alt="T"), "tumor"),
         somatic_genotype("2", dict(tumor=(0.9, 0, 0, 0, 0), gq=3, locus=100, ref="G", alt=""), "tumor")]
    out = tmp_path / name
    check_output_path(str(out))
    _write_genotypes(str(out), g, parquet=dict(part_of=[0, 2, 2, 2], n_parts=4))
    files = sorted(os.listdir(out))
    assert files == ["_SUCCESS", "_common_metadata", "_metadata", "part-r-00000.gz.parquet",
                     "part-r-00001.gz.parquet", "part-r-00002.gz.parquet", "part-r-00003.gz.parquet"]
    _same_records(read_parquet_dir(str(out)), _plain_from_json(g))
    with pytest.raises(OutputFormatError, match="already exists"):
        check_output_path(str(out))
    for codec, ext in (("SNAPPY", ".snappy"), ("UNCOMPRESSED", "")):
        d = tmp_path / (codec + ".adam")
        _write_genotypes(str(d), g, parquet=dict(codec=codec, dictionary=False))
        assert "part-r-00000%s.parquet" % ext in os.listdir(d)
        _same_records(read_parquet_dir(str(d)), _plain_from_json(g))
    with pytest.raises(OutputFormatError, match="LZO"):
        check_output_path(str(tmp_path / "z.adam"), "LZO")


def test_parquet_footer_carries_the_avro_schema(tmp_path):
    import pyarrow.parquet as pq
    from guacamole_amd.output import write_parquet_dir
    f = write_parquet_dir(str(tmp_path / "a.adam"), [germline_genotype("1", 5, "x", ("Alt", "Alt"), "C", "G")])[0]
    meta = pq.read_metadata(f).metadata
    sch = json.loads(meta[b"parquet.avro.schema"])
    assert sch["name"] == "Genotype" and sch["namespace"] == "org.bdgenomics.formats.avro"
    assert [x["name"] for x in sch["fields"]][:6] == ["variant", "variantCallingAnnotations", "sampleId",
                                                      "sampleDescription", "processingDescription", "alleles"]
    alleles = next(x for x in sch["fields"] if x["name"] == "alleles")["type"]["items"]
    assert alleles["symbols"] == ["Ref", "Alt", "OtherAlt", "NoCall"]


def test_parquet_parts_follow_the_loci_tasks():
    """Records go to the part of the loci task whose range holds them (flatten_partitions order)."""
    import argparse
    from guacamole_amd.commands import parquet_options
    args = argparse.Namespace(parquet_compression_codec="GZIP", parquet_page_size=1 << 20,
                              parquet_block_size=128 << 20, parquet_disable_dictionary=False)
    flat = (np.array([0, 0, 1]), np.array([0, 100, 0]), np.array([100, 200, 50]), np.array([0, 1, 2]))
    o = parquet_options(args, flat, {"a": 0, "b": 1}, ["a", "a", "a", "b"], [0, 99, 150, 10])
    assert o["part_of"].tolist() == [0, 0, 1, 2] and o["n_parts"] == 3


def test_default_parallelism_is_the_rank_count(monkeypatch):
    """--parallelism 0 = sc.defaultParallelism (DistributedUtil.scala:59): the rank count here."""
    from guacamole_amd.commands import single_process_only, task_count
    assert task_count(0, 1) == 1 and task_count(0, 4) == 4 and task_count(7, 4) == 7
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(RuntimeError, match="single process"):
        single_process_only("variant-support")
