"""Host-side timing of the region plan (gq_bam_dev_plan, no BAI: host probes) on the configs[3]
rank-7 layout at a reduced depth (CPU only: the plan needs no GPU).  usage: python
scripts/plan_timing.py [depth]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import genome_parts, merged_pieces  # noqa: E402
from guacamole_amd import synthetic  # noqa: E402
from guacamole_amd.bamdev import MappedBam  # noqa: E402
from guacamole_amd.genomes import B37  # noqa: E402
from guacamole_amd.loci import LociMapBuilder, LociSet  # noqa: E402

depth = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
parts, _ = genome_parts(8, True)
mine = [p for p in parts if p[4] == 7]
pieces = merged_pieces(mine)
first = mine[0]
gen = [(c, ln, max(0, s - 5_000_000) if c == first[0] else s, e) for c, ln, s, e in pieces]
g = synthetic.generate_pieces(gen, depth, seed=synthetic.SEED + 4)
path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gq_plan_%d.bam" % os.getpid())
try:
    g.write_bam(path, level=1, dictionary=list(B37))
    print("reads", g.n, "bam bytes", os.path.getsize(path), flush=True)
    del g
    b = LociMapBuilder()
    for c, _, s, e in pieces:
        b.put(c, int(s), int(e), 0)
    region = LociSet(b.result())
    for rep in range(2):
        t = time.perf_counter()
        m = MappedBam(path, populate=False)
        t1 = time.perf_counter()
        info = m.plan(region, 1 << 20, None)
        t2 = time.perf_counter()
        print("map %.3f s  plan %.3f s  probes %d  segments %d  blocks %d" % (t1 - t, t2 - t1, info["probes"],
                                                                              info["n_segments"], info["n_blocks"]))
        m.close()
finally:
    os.remove(path)
