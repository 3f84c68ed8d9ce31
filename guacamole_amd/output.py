"""Genotype output: bdg-formats Genotype records, Avro-JSON and VCF writers, dbSNP join.

Restates the record builders the two callers use (paths relative to
/root/reference/src/main/scala/org/hammerlab/guacamole/):
  * germline: Genotype{alleles, sampleId, variant{start, referenceAllele, alternateAllele,
    contig{contigName}}} — no `end`, no depths (commands/GermlineThresholdCaller.scala:106-117)
  * somatic: AlleleConversions.calledSomaticAlleleToADAMGenotype
    (variants/AlleleConversions.scala:47-62): alleles [Ref, Alt], GQ = phredScaledSomaticLikelihood,
    readDepth / alternateReadDepth from the tumor evidence, referenceReadDepth = DP - alt,
    expectedAlleleDosage = alt / DP (float32), variant = CalledSomaticAllele.adamVariant
    (variants/ReferenceVariant.scala:42-48) whose end is start + 1 (CalledSomaticAllele.scala:46)
  * dbSNP join: SomaticStandardCaller.scala:139-149 (leftOuterJoin on the ADAM Variant)
The writer path (Common.writeVariantsFromArguments, Common.scala:246-304) picks JSON for
"" / ".json" and VCF for ".vcf".  JSON is what Avro's JsonEncoder writes for the Genotype schema
through Jackson's default pretty printer: every schema field in schema order, nullable fields as
unions ({"<type>": value} or null).  The schema is bdg-formats 0.6.1 (pom.xml:20), a dependency
absent from /root/reference: its field lists are restated below from the published schema and are
parity unpinned, as is ADAM 0.18's VCF rendering (saveAsVcf).
"""
from __future__ import annotations

import json
import math
import sys
from typing import Dict, Iterable, List, Optional, Sequence, TextIO, Tuple

import numpy as np

GT_CODE = {"Ref": "0", "Alt": "1", "OtherAlt": ".", "NoCall": "."}

_NS = "org.bdgenomics.formats.avro."
# bdg-formats 0.6.1 records (field, Avro type, default); "?T" = union {null, T} default null,
# "T?" = union {T, null} with the default shown, "[T]" = array (default [])
CONTIG_SCHEMA: List[Tuple[str, str, object]] = [
    ("contigName", "?string", None), ("contigLength", "?long", None), ("contigMD5", "?string", None),
    ("referenceURL", "?string", None), ("assembly", "?string", None), ("species", "?string", None),
    ("referenceIndex", "?int", None)]
VARIANT_SCHEMA: List[Tuple[str, str, object]] = [
    ("contig", "?Contig", None), ("start", "?long", None), ("end", "?long", None),
    ("referenceAllele", "?string", None), ("alternateAllele", "?string", None),
    ("svAllele", "?StructuralVariant", None), ("isSomatic", "boolean?", False)]
GENOTYPE_SCHEMA: List[Tuple[str, str, object]] = [
    ("variant", "?Variant", None), ("variantCallingAnnotations", "?VariantCallingAnnotations", None),
    ("sampleId", "?string", None), ("sampleDescription", "?string", None),
    ("processingDescription", "?string", None), ("alleles", "[GenotypeAllele]", []),
    ("expectedAlleleDosage", "?float", None), ("referenceReadDepth", "?int", None),
    ("alternateReadDepth", "?int", None), ("readDepth", "?int", None), ("minReadDepth", "?int", None),
    ("genotypeQuality", "?int", None), ("genotypeLikelihoods", "[float]", []),
    ("nonReferenceLikelihoods", "[float]", []), ("strandBiasComponents", "[int]", []),
    ("splitFromMultiAllelic", "boolean?", False), ("isPhased", "?boolean", None), ("phaseSetId", "?int", None),
    ("phaseQuality", "?int", None)]
_RECORDS = {"Contig": CONTIG_SCHEMA, "Variant": VARIANT_SCHEMA, "Genotype": GENOTYPE_SCHEMA}
# Records the callers never set (always null in their output) but which the Parquet schema still
# carries as groups: restated from bdg-formats 0.6.1, parity unpinned like the rest
STRUCTURAL_VARIANT_SCHEMA: List[Tuple[str, str, object]] = [
    ("type", "?StructuralVariantType", None), ("assembly", "?string", None), ("precise", "boolean?", True),
    ("startWindow", "?int", None), ("endWindow", "?int", None)]
ANNOTATIONS_SCHEMA: List[Tuple[str, str, object]] = [
    ("variantIsPassing", "?boolean", None), ("variantFilters", "[string]", []), ("downsampled", "?boolean", None),
    ("baseQRankSum", "?float", None), ("fisherStrandBiasPValue", "?float", None), ("rmsMapQ", "?float", None),
    ("mapq0Reads", "?int", None), ("mqRankSum", "?float", None), ("readPositionRankSum", "?float", None),
    ("genotypePriors", "[float]", []), ("genotypePosteriors", "[float]", []), ("vqslod", "?float", None),
    ("culprit", "?string", None), ("attributes", "{string}", {})]
_ENUMS = {"GenotypeAllele": ["Ref", "Alt", "OtherAlt", "NoCall"],
          "StructuralVariantType": ["DELETION", "INSERTION", "INVERSION", "MOBILE_INSERTION", "MOBILE_DELETION",
                                    "DUPLICATION", "TANDEM_DUPLICATION"]}
# The reads' record (adam.py: ADAM AlignmentRecord input, Read.scala:454-539), bdg-formats 0.6.1
# as restated here (readNum in place of the older firstOfPair / secondOfPair), parity unpinned
ALIGNMENT_RECORD_SCHEMA: List[Tuple[str, str, object]] = [
    ("contig", "?Contig", None), ("start", "?long", None), ("oldPosition", "?long", None), ("end", "?long", None),
    ("mapq", "?int", None), ("readName", "?string", None), ("sequence", "?string", None), ("qual", "?string", None),
    ("cigar", "?string", None), ("oldCigar", "?string", None), ("basesTrimmedFromStart", "int?", 0),
    ("basesTrimmedFromEnd", "int?", 0), ("readPaired", "boolean?", False), ("properPair", "boolean?", False),
    ("readMapped", "boolean?", False), ("mateMapped", "boolean?", False), ("readNum", "int?", 0),
    ("failedVendorQualityChecks", "boolean?", False), ("duplicateRead", "boolean?", False),
    ("readNegativeStrand", "boolean?", False), ("mateNegativeStrand", "boolean?", False),
    ("primaryAlignment", "boolean?", False), ("secondaryAlignment", "boolean?", False),
    ("supplementaryAlignment", "boolean?", False), ("mismatchingPositions", "?string", None),
    ("origQual", "?string", None), ("attributes", "?string", None), ("recordGroupName", "?string", None),
    ("recordGroupSequencingCenter", "?string", None), ("recordGroupDescription", "?string", None),
    ("recordGroupRunDateEpoch", "?long", None), ("recordGroupFlowOrder", "?string", None),
    ("recordGroupKeySequence", "?string", None), ("recordGroupLibrary", "?string", None),
    ("recordGroupPredictedMedianInsertSize", "?int", None), ("recordGroupPlatform", "?string", None),
    ("recordGroupPlatformUnit", "?string", None), ("recordGroupSample", "?string", None),
    ("mateAlignmentStart", "?long", None), ("mateAlignmentEnd", "?long", None), ("mateContig", "?Contig", None),
    ("inferredInsertSize", "?long", None)]
_ALL_RECORDS = dict(_RECORDS, StructuralVariant=STRUCTURAL_VARIANT_SCHEMA,
                    VariantCallingAnnotations=ANNOTATIONS_SCHEMA, AlignmentRecord=ALIGNMENT_RECORD_SCHEMA)


def germline_genotype(contig: str, start: int, sample: str, alleles, ref: str, alt: str) -> Dict:
    """GermlineThresholdCaller.scala:106-117 (the fields the builder sets)."""
    return dict(alleles=list(alleles), sampleId=sample,
                variant=dict(start=int(start), referenceAllele=ref, alternateAllele=alt,
                             contig=dict(contigName=contig)))


def somatic_genotype(contig: str, row: Dict, sample: str) -> Dict:
    """AlleleConversions.calledSomaticAlleleToADAMGenotype (AlleleConversions.scala:47-62)."""
    t = row["tumor"]  # (likelihood, readDepth, alleleReadDepth, forwardDepth, alleleForwardDepth, ...)
    depth, alt_depth = int(t[1]), int(t[2])
    with np.errstate(divide="ignore", invalid="ignore"):
        dosage = float(np.float32(alt_depth) / np.float32(depth))
    return dict(alleles=["Ref", "Alt"], sampleId=sample, genotypeQuality=int(row["gq"]), readDepth=depth,
                expectedAlleleDosage=dosage, referenceReadDepth=depth - alt_depth, alternateReadDepth=alt_depth,
                variant=dict(start=int(row["locus"]), end=int(row["locus"]) + 1, referenceAllele=row["ref"],
                             alternateAllele=row["alt"], contig=dict(contigName=contig)))


def called_allele_genotype(contig: str, row: Dict, sample: str) -> Dict:
    """AlleleConversions.calledAlleleToADAMGenotype (AlleleConversions.scala:30-45): as the
    somatic builder with GQ = the evidence's phredScaledLikelihood (CalledAllele.scala:39: end
    = start + 1)."""
    return somatic_genotype(contig, row, sample)


# ---- Avro JSON encoding -------------------------------------------------------------------
def java_float(x: float) -> str:
    """Float.toString of a float32 (what Jackson writes for JsonEncoder.writeFloat): the shortest
    repr that round-trips the float32, "d.ddd" for 1e-3 <= |x| < 1e7, else "d.dddE<exp>"."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    f = np.float32(x)
    if f == 0:
        return "-0.0" if math.copysign(1.0, float(f)) < 0 else "0.0"
    s = np.format_float_scientific(f, unique=True, trim="-")  # e.g. '2e-01', '1.2345e+07'
    mant, exp = s.split("e")
    e = int(exp)
    neg = mant.startswith("-")
    digits = mant.lstrip("-").replace(".", "")
    if 1e-3 <= abs(float(f)) < 1e7:
        if e >= 0:
            ip = digits[:e + 1].ljust(e + 1, "0")
            fp = digits[e + 1:] or "0"
        else:
            ip, fp = "0", "0" * (-e - 1) + digits
        out = ip + "." + fp
    else:
        out = digits[0] + "." + (digits[1:] or "0") + "E" + str(e)
    return ("-" if neg else "") + out


def avro_datum(record: str, value: Optional[Dict]) -> Dict:
    """The JsonEncoder's view of a record: every schema field in order, unions wrapped."""
    value = value or {}
    out: Dict = {}
    for name, typ, default in _RECORDS[record]:
        v = value.get(name, default)
        if typ.startswith("["):
            out[name] = list(v)
        elif v is None:
            out[name] = None
        else:
            base = typ.strip("?")
            if base in _RECORDS:
                out[name] = {_NS + base: avro_datum(base, v)}
            else:
                out[name] = {base: v}
    return out


def _pretty(v, ind: int, float_fields: bool = False) -> str:
    """Jackson 1.x DefaultPrettyPrinter: objects one field a line ("name" : value) at two-space
    indents, arrays inline ([ a, b ]), empty containers "{ }" / "[ ]"."""
    if isinstance(v, dict):
        if not v:
            return "{ }"
        pad = "  " * (ind + 1)
        items = []
        for k, x in v.items():
            items.append(pad + json.dumps(k) + " : " + _pretty(x, ind + 1, k == "float"))
        return "{\n" + ",\n".join(items) + "\n" + "  " * ind + "}"
    if isinstance(v, list):
        return "[ " + ", ".join(_pretty(x, ind) for x in v) + " ]" if v else "[ ]"
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        return "null"
    if float_fields or isinstance(v, float):
        return java_float(float(v))
    return json.dumps(v)


def avro_json(genotypes: Iterable[Dict]) -> str:
    """The bytes Common.writeVariantsFromArguments writes for JSON output (Common.scala:263-285):
    the records, pretty-printed and separated by Jackson's root separator (one space), then a
    newline."""
    return " ".join(_pretty(avro_datum("Genotype", g), 0) for g in genotypes) + "\n"


def read_avro_json(text: str) -> List[Dict]:
    """The records of an avro_json text (whitespace-separated JSON objects)."""
    dec, i, out = json.JSONDecoder(), 0, []
    n = len(text)
    while True:
        while i < n and text[i] in " \t\r\n":
            i += 1
        if i >= n:
            return out
        obj, i = dec.raw_decode(text, i)
        out.append(obj)


def write_json(path: str, genotypes: Iterable[Dict]) -> None:
    out: TextIO = open(path, "w") if path else sys.stdout
    try:
        out.write(avro_json(genotypes))
    finally:
        if path:
            out.close()


VCF_PART = "part-r-00000"


def write_vcf_dir(path: str, genotypes: List[Dict], contig_lengths: Optional[Dict[str, int]] = None) -> str:
    """saveAsVcf after coalesce(1, shuffle = true) (Common.scala:293): Hadoop's new-API output
    layout — the directory `path` holding the single part file part-r-00000 and the committer's
    empty _SUCCESS marker.  Returns the part file's path."""
    import os
    os.makedirs(path, exist_ok=False)
    part = os.path.join(path, VCF_PART)
    write_vcf(part, genotypes, contig_lengths)
    open(os.path.join(path, "_SUCCESS"), "w").close()
    return part


# ---- ADAM Parquet (adamParquetSave) -------------------------------------------------------
# parquet-mr names a part file getDefaultWorkFile(codec extension + ".parquet")
PARQUET_CODECS = {"UNCOMPRESSED": ("none", ""), "SNAPPY": ("snappy", ".snappy"), "GZIP": ("gzip", ".gz")}


def avro_schema(record: str = "Genotype", _seen=None) -> Dict:
    """The Avro schema of a restated bdg-formats record, as parquet-avro stores it in the
    footer (key "parquet.avro.schema"): named types spelled out at first use, then by name."""
    seen = set() if _seen is None else _seen
    seen.add(record)

    def typ(t: str):
        if t.startswith("["):
            return {"type": "array", "items": typ(t[1:-1])}
        if t.startswith("{"):
            return {"type": "map", "values": typ(t[1:-1])}
        base = t.strip("?")
        if base in _ALL_RECORDS:
            inner = _NS + base if base in seen else avro_schema(base, seen)
        elif base in _ENUMS:
            inner = _NS + base if base in seen else {"type": "enum", "name": base, "namespace": _NS[:-1],
                                                     "symbols": _ENUMS[base]}
            seen.add(base)
        else:
            inner = base
        if t.startswith("?"):
            return ["null", inner]
        if t.endswith("?"):
            return [inner, "null"]
        return inner
    fields = [{"name": n, "type": typ(t), "default": d} for n, t, d in _ALL_RECORDS[record]]
    return {"type": "record", "name": record, "namespace": _NS[:-1], "fields": fields}


def _arrow_type(t: str):
    """parquet-avro's mapping of an Avro type (AvroSchemaConverter): a union with null is an
    optional column, records groups, enums and strings UTF8 binaries, arrays and maps required."""
    import pyarrow as pa
    if t.startswith("["):
        return pa.list_(pa.field("array", _arrow_type(t[1:-1]), nullable=False))
    if t.startswith("{"):
        return pa.map_(pa.string(), pa.field("value", _arrow_type(t[1:-1]), nullable=False))
    base = t.strip("?")
    if base in _ALL_RECORDS:
        return pa.struct(_arrow_fields(base))
    if base in _ENUMS or base == "string":
        return pa.string()
    return {"long": pa.int64(), "int": pa.int32(), "float": pa.float32(), "boolean": pa.bool_()}[base]


def _arrow_fields(record: str):
    import pyarrow as pa
    return [pa.field(n, _arrow_type(t), nullable="?" in t) for n, t, _ in _ALL_RECORDS[record]]


def plain_record(record: str, value: Optional[Dict]) -> Dict:
    """Every schema field of a record in schema order with its default filled in (no union
    wrappers): the row parquet-avro writes for a builder that set only some fields."""
    out: Dict = {}
    value = value or {}
    for name, typ, default in _ALL_RECORDS[record]:
        v = value.get(name, default)
        base = typ.strip("?")
        if typ.startswith("["):
            v = list(v)
        elif typ.startswith("{"):
            v = dict(v)
        elif v is not None and base in _ALL_RECORDS:
            v = plain_record(base, v)
        out[name] = v
    return out


def unwrap_avro_json(record: str, datum: Optional[Dict]) -> Optional[Dict]:
    """A record read back from avro_json (unions wrapped as {"<type>": value}) as plain_record
    shapes it, so the two writers' outputs compare field for field."""
    if datum is None:
        return None
    out: Dict = {}
    for name, typ, _ in _ALL_RECORDS[record]:
        v = datum[name]
        base = typ.strip("?")
        if isinstance(v, dict) and not typ.startswith("{") and len(v) == 1:
            (k, v), = v.items()
        if v is not None and base in _ALL_RECORDS:
            v = unwrap_avro_json(base, v)
        out[name] = v
    return out


def write_parquet_dir(path: str, genotypes: List[Dict], part_of: Optional[Sequence[int]] = None, n_parts: int = 1,
                      codec: str = "GZIP", page_size: int = 1 << 20, block_size: int = 128 << 20,
                      dictionary: bool = True, record: str = "Genotype") -> List[str]:
    """adamParquetSave (Common.scala:294-302; ADAM 0.18 rdd.map((null, _)).saveAsNewAPIHadoopFile
    through AvroParquetOutputFormat) for Genotype records: the Hadoop output directory `path`
    with one part-r-NNNNN<codec>.parquet per RDD partition (record i goes to part part_of[i]; the
    callers' genotypes RDD has one partition per loci task, empty ones still written), the
    summary files _metadata / _common_metadata, and _SUCCESS.  Options are ParquetArgs'
    (-parquet_compression_codec GZIP, -parquet_page_size 1 MiB, -parquet_block_size 128 MiB,
    dictionary encoding on).  The schema is the restated bdg-formats Genotype (or `record`, e.g.
    AlignmentRecord for adam.write_alignment_parquet), with the Avro schema in the footer; byte
    parity with parquet-mr's files is unpinned."""
    import os
    import pyarrow as pa
    import pyarrow.parquet as pq
    if codec not in PARQUET_CODECS:
        raise ValueError("-parquet_compression_codec %s is not available (one of %s)"
                         % (codec, ", ".join(sorted(PARQUET_CODECS))))
    comp, ext = PARQUET_CODECS[codec]
    schema = pa.schema(_arrow_fields(record),
                       metadata={"parquet.avro.schema": json.dumps(avro_schema(record)), "writer.model.name": "avro"})
    os.makedirs(path, exist_ok=False)
    part_of = np.zeros(len(genotypes), np.int64) if part_of is None else np.asarray(part_of, np.int64)
    n_parts = max(1, int(n_parts), int(part_of.max()) + 1 if len(part_of) else 1)
    order = np.argsort(part_of, kind="stable")
    bounds = np.searchsorted(part_of[order], np.arange(n_parts + 1))
    collector, files = [], []
    for p in range(n_parts):
        rows = [plain_record(record, genotypes[i]) for i in order[bounds[p]:bounds[p + 1]]]
        table = pa.Table.from_pylist(rows, schema=schema)
        per_row = table.nbytes / max(1, table.num_rows)
        name = "part-r-%05d%s.parquet" % (p, ext)
        pq.write_table(table, os.path.join(path, name), compression=comp, data_page_size=int(page_size),
                       use_dictionary=bool(dictionary), row_group_size=max(1, int(block_size / max(1.0, per_row))),
                       use_compliant_nested_type=False, metadata_collector=collector)
        collector[-1].set_file_path(name)
        files.append(os.path.join(path, name))
    pq.write_metadata(schema, os.path.join(path, "_common_metadata"), use_compliant_nested_type=False)
    pq.write_metadata(schema, os.path.join(path, "_metadata"), metadata_collector=collector,
                      use_compliant_nested_type=False)
    open(os.path.join(path, "_SUCCESS"), "w").close()
    return files


def read_parquet_dir(path: str) -> List[Dict]:
    """The Genotype rows of a write_parquet_dir directory, part files in name order (maps as
    dicts)."""
    import glob
    import os
    import pyarrow.parquet as pq
    out: List[Dict] = []

    def fix(record: str, v):
        for name, typ, _ in _ALL_RECORDS[record]:
            base = typ.strip("?")
            if typ.startswith("{"):
                v[name] = dict(v[name])
            elif v[name] is not None and base in _ALL_RECORDS:
                fix(base, v[name])
        return v
    for f in sorted(glob.glob(os.path.join(path, "part-r-*.parquet"))):
        out.extend(fix("Genotype", r) for r in pq.read_table(f).to_pylist())
    return out


def write_vcf(path: str, genotypes: List[Dict], contig_lengths: Optional[Dict[str, int]] = None) -> None:
    """One VCF line per Genotype (VCF 4.1; POS is 1-based = start + 1) into the file `path`."""
    def fields(g):
        v = g["variant"]
        fmt, vals = "GT", "/".join(GT_CODE.get(a, ".") for a in g["alleles"])
        if "genotypeQuality" in g:
            fmt += ":GQ:DP:AD"
            vals += ":%d:%d:%d,%d" % (g["genotypeQuality"], g["readDepth"], g["referenceReadDepth"],
                                       g["alternateReadDepth"])
        return (v["contig"]["contigName"], v["start"], v["referenceAllele"], v["alternateAllele"], g["sampleId"],
                fmt, vals)
    _write_vcf_fields(path, [fields(g) for g in genotypes], contig_lengths)


def write_vcf_dir_germline(path: str, rows, sample_name, contig_lengths: Optional[Dict[str, int]] = None) -> str:
    """write_vcf_dir for germline-threshold rows (contig, locus, sample slot, (gt0, gt1), ref, alt, ...)
    straight from the caller's columns: the lines write_vcf writes for their germline_genotype
    records (GermlineThresholdCaller.scala:106-117 sets alleles, sample, variant only)."""
    import os
    os.makedirs(path, exist_ok=False)
    part = os.path.join(path, VCF_PART)
    gt = {(a, b): GT_CODE.get(a, ".") + "/" + GT_CODE.get(b, ".") for a in GT_CODE for b in GT_CODE}
    _write_vcf_fields(part, [(c, l, ref, alt, sample_name(s), "GT", gt[g]) for c, l, s, g, ref, alt, *_ in rows],
                      contig_lengths)
    open(os.path.join(path, "_SUCCESS"), "w").close()
    return part


def write_vcf_dir_germline_calls(path: str, calls, contig_names, sample_name, contig_lengths=None) -> str:
    """write_vcf_dir_germline straight from a GermlineCalls' columns: records of one sample (the
    common case) go through the library's line writer (gq_write_vcf_germline) without a Python
    object per record; several samples take write_vcf_dir_germline's layout."""
    import os
    import numpy as np
    from . import native
    slots = np.unique(calls.a["sample"]) if len(calls) else np.zeros(0, np.uint8)
    names = sorted({sample_name(int(s)) for s in slots})
    if len(names) > 1:
        return write_vcf_dir_germline(path, calls.tuples(contig_names), sample_name, contig_lengths)
    os.makedirs(path, exist_ok=False)
    part = os.path.join(path, VCF_PART)
    native.write_vcf_germline(part, vcf_header(names, contig_lengths), calls, contig_names)
    open(os.path.join(path, "_SUCCESS"), "w").close()
    return part


def vcf_header(samples, contig_lengths: Optional[Dict[str, int]]) -> str:
    """The ## lines and the #CHROM line over `samples` (sample columns in order)."""
    out = ["##fileformat=VCFv4.1\n",
           '##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">\n',
           '##FORMAT=<ID=GQ,Number=1,Type=Integer,Description="Genotype Quality">\n',
           '##FORMAT=<ID=DP,Number=1,Type=Integer,Description="Read Depth">\n',
           '##FORMAT=<ID=AD,Number=R,Type=Integer,Description="Allelic depths (ref, alt)">\n']
    for c, ln in (contig_lengths or {}).items():
        out.append("##contig=<ID=%s,length=%d>\n" % (c, ln))
    out.append("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples) + "\n")
    return "".join(out)


def _write_vcf_fields(path: str, recs, contig_lengths: Optional[Dict[str, int]]) -> None:
    """recs: (contig, start, ref, alt, sampleId, FORMAT, values) per genotype, in output order."""
    samples: Dict[str, int] = {}
    for r in recs:
        if r[4] not in samples:
            samples[r[4]] = len(samples)
    ns = len(samples)
    out = [vcf_header(samples, contig_lengths)]
    if ns == 1:
        out.extend("%s\t%d\t.\t%s\t%s\t.\t.\t.\t%s\t%s\n" % (c, s + 1, ref, alt, fmt, vals)
                   for c, s, ref, alt, _, fmt, vals in recs)
    else:
        for c, s, ref, alt, sid, fmt, vals in recs:
            cols = ["."] * ns
            cols[samples[sid]] = vals
            out.append("%s\t%d\t.\t%s\t%s\t.\t.\t.\t%s\t%s\n" % (c, s + 1, ref, alt, fmt, "\t".join(cols)))
    with open(path, "w") as fh:
        fh.write("".join(out))


# ---- dbSNP annotation join ----------------------------------------------------------------
def read_dbsnp_vcf(path: str) -> List[Dict]:
    """ADAMContext.loadVariantAnnotations over a VCF, restated as what the join reads: one
    entry per (record, ALT allele) with the variant key (contig, 0-based start, end = start +
    len(REF), REF, ALT) and the numeric dbSNP id of an "rs<N>" ID column (None otherwise)."""
    import gzip
    with open(path, "rb") as fh:
        gz = fh.read(2) == b"\x1f\x8b"
    out: List[Dict] = []
    with (gzip.open(path, "rt") if gz else open(path)) as fh:
        for line in fh:
            if not line.strip() or line.startswith("#"):
                continue
            f = line.rstrip("\n").split("\t")
            if len(f) < 5:
                raise ValueError("%s: malformed VCF line: %r" % (path, line[:80]))
            contig, pos, vid, ref = f[0], int(f[1]) - 1, f[2], f[3]
            rs = None
            for tok in vid.split(";"):
                if tok.startswith("rs") and tok[2:].isdigit():
                    rs = int(tok[2:])
                    break
            for alt in f[4].split(","):
                out.append(dict(contig=contig, start=pos, end=pos + len(ref), ref=ref, alt=alt, rs_id=rs))
    return out


def dbsnp_join(rows: List[Dict], dbsnp: List[Dict]) -> List[Dict]:
    """potentialGenotypes.keyBy(_.adamVariant).leftOuterJoin(dbSnp.keyBy(_.getVariant))
    (SomaticStandardCaller.scala:141-147): each call gets rs_id from every dbSNP entry with its
    variant key (the call repeated once per match, as a join does), None when none matches.
    The reference's post-shuffle record order is Spark hash-partition order; calls keep theirs."""
    index: Dict[tuple, List[Optional[int]]] = {}
    for d in dbsnp:
        index.setdefault((d["contig"], d["start"], d["end"], d["ref"], d["alt"]), []).append(d["rs_id"])
    out = []
    for r in rows:
        key = (r["contig"], int(r["locus"]), int(r["locus"]) + 1, r["ref"], r["alt"])
        for rs in index.get(key, [None]):
            x = dict(r)
            x["rs_id"] = rs
            out.append(x)
    return out
