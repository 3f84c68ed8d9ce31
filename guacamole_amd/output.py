"""Genotype output: bdg-formats Genotype records as JSON lines and a VCF writer.

Restates the record builders the two callers use:
  * germline: Genotype{alleles, sampleId, variant{contig, start, end, ref, alt}}
    (commands/GermlineThresholdCaller.scala:106-117)
  * somatic: AlleleConversions.calledSomaticAlleleToADAMGenotype
    (variants/AlleleConversions.scala:47-62): GQ = phredScaledSomaticLikelihood, DP / AD
    from the tumor evidence, expectedAlleleDosage = alt / DP (float32).
The writer path (Common.writeVariantsFromArguments, Common.scala:246-304) picks JSON for
"" / ".json" and VCF for ".vcf".  ADAM's exact VCF rendering (saveAsVcf) and the Avro
JSON encoder's field order are third-party behaviour that is parity unpinned;
the fields and values written here are the reference's.
"""
from __future__ import annotations

import json
import sys
from typing import Dict, Iterable, List, Optional, TextIO

GT_CODE = {"Ref": "0", "Alt": "1", "OtherAlt": ".", "NoCall": "."}


def germline_genotype(contig: str, start: int, sample: str, alleles, ref: str, alt: str) -> Dict:
    return dict(alleles=list(alleles), sampleId=sample,
                variant=dict(contig=dict(contigName=contig), start=int(start), end=int(start) + len(ref),
                             referenceAllele=ref, alternateAllele=alt))


def somatic_genotype(contig: str, row: Dict, sample: str) -> Dict:
    t = row["tumor"]  # (likelihood, readDepth, alleleReadDepth, forwardDepth, alleleForwardDepth, ...)
    depth, alt_depth = int(t[1]), int(t[2])
    import numpy as np
    return dict(alleles=["Ref", "Alt"], sampleId=sample, genotypeQuality=int(row["gq"]), readDepth=depth,
                expectedAlleleDosage=float(np.float32(alt_depth) / np.float32(depth)) if depth else float("nan"),
                referenceReadDepth=depth - alt_depth, alternateReadDepth=alt_depth,
                variant=dict(contig=dict(contigName=contig), start=int(row["locus"]),
                             end=int(row["locus"]) + len(row["ref"]), referenceAllele=row["ref"],
                             alternateAllele=row["alt"]))


def write_json(path: str, genotypes: Iterable[Dict]) -> None:
    out: TextIO = open(path, "w") if path else sys.stdout
    try:
        for g in genotypes:
            out.write(json.dumps(g) + "\n")
    finally:
        if path:
            out.close()


def write_vcf(path: str, genotypes: List[Dict], contig_lengths: Optional[Dict[str, int]] = None) -> None:
    """One VCF line per Genotype (VCF 4.1; POS is 1-based = start + 1)."""
    samples: List[str] = []
    for g in genotypes:
        if g["sampleId"] not in samples:
            samples.append(g["sampleId"])
    with open(path, "w") as fh:
        fh.write("##fileformat=VCFv4.1\n")
        fh.write('##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">\n')
        fh.write('##FORMAT=<ID=GQ,Number=1,Type=Integer,Description="Genotype Quality">\n')
        fh.write('##FORMAT=<ID=DP,Number=1,Type=Integer,Description="Read Depth">\n')
        fh.write('##FORMAT=<ID=AD,Number=R,Type=Integer,Description="Allelic depths (ref, alt)">\n')
        for c, ln in (contig_lengths or {}).items():
            fh.write("##contig=<ID=%s,length=%d>\n" % (c, ln))
        fh.write("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples) + "\n")
        for g in genotypes:
            v = g["variant"]
            fmt, vals = ["GT"], ["/".join(GT_CODE.get(a, ".") for a in g["alleles"])]
            if "genotypeQuality" in g:
                fmt += ["GQ", "DP", "AD"]
                vals += [str(g["genotypeQuality"]), str(g["readDepth"]),
                         "%d,%d" % (g["referenceReadDepth"], g["alternateReadDepth"])]
            cols = ["."] * len(samples)
            cols[samples.index(g["sampleId"])] = ":".join(vals)
            fh.write("\t".join([v["contig"]["contigName"], str(v["start"] + 1), ".", v["referenceAllele"],
                                v["alternateAllele"], ".", ".", ".", ":".join(fmt)] + cols) + "\n")
