"""Diagnostics for germline_direct on chrM (round 6): the records of the direct kernel vs the
oracle, with the library's error text if a call fails."""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from conftest import fixture  # noqa: E402
from guacamole_amd import native  # noqa: E402
from guacamole_amd.commands import device_reads  # noqa: E402
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly  # noqa: E402
from guacamole_amd.reads import InputFilters, load_reads  # noqa: E402
from guacamole_amd.synthetic import generate  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(ctx, rs, name):
    loci = flatten_partitions(partition_loci_uniformly(1, LociSet.parse("all").result(rs.contig_lengths_map)),
                              rs.contig_index())
    d = device_reads(ctx, rs)
    try:
        got = ctx.germline_threshold(d, loci, 8).tuples(rs.contig_names)
    except Exception:
        traceback.print_exc()
        print(name, "FAILED", flush=True)
        return False
    want = O.germline_threshold(rs, loci, 8)
    tm = ctx.timings()
    print(name, "records", len(got), "oracle", len(want), "equal", got == want, "walk_tiles", tm["walk_tiles"],
          "tiles", tm["tiles"], flush=True)
    return got == want


ctx = native.Context(0)
g = generate(100_000, 30, seed=7, indel_rate=3e-4)
ok = run(ctx, g.to_read_set(), "synthetic30x")
g5 = generate(12_000, 500.0, seed=5, indel_rate=3e-4)
ok = run(ctx, g5.to_read_set(), "synthetic500x") and ok
chrm = load_reads(fixture("chrM.sorted.bam"), InputFilters.make(mapped=True, non_duplicate=True, has_md_tag=True))
ok = run(ctx, chrm, "chrM") and ok
sys.exit(0 if ok else 1)
