#!/usr/bin/env python3
"""Diff the somatic calls of two library builds on the bench's tumor/normal shard, and check
the loci where they differ against the CPU oracle (small windows around each).

  python scripts/somatic_diff.py OLD.so NEW.so [--length L]
Each build runs in its own process (GQ_LIB); the calls go through JSON files in gpurun_out/."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CHR20 = 63_025_520


def run_one(out):
    from guacamole_amd import native, synthetic
    L = int(os.environ.get("SD_LENGTH", CHR20))
    seed = synthetic.SEED + 3
    tg = synthetic.generate(L, 60.0, seed=seed, somatic_rate=2e-4, tumor=True, read_seed=11)
    ng = synthetic.generate(L, 30.0, seed=seed, somatic_rate=2e-4, tumor=False, read_seed=12)
    ctx = native.Context(0)
    t, n = ctx.upload(tg.arrays), ctx.upload(ng.arrays)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([L - 1], np.int64), np.array([0], np.int64))
    c = ctx.somatic_standard(t, n, loci)
    rows = [[r["locus"], r["ref"], r["alt"], r["log_odds"], r["gq"], r["flags"]] for r in c.rows]
    json.dump(rows, open(out, "w"))


def main():
    if sys.argv[1] == "--one":
        run_one(sys.argv[2])
        return
    old, new = sys.argv[1], sys.argv[2]
    os.makedirs("gpurun_out", exist_ok=True)
    for lib, out in ((old, "gpurun_out/sd_old.json"), (new, "gpurun_out/sd_new.json")):
        subprocess.check_call([sys.executable, __file__, "--one", out], env=dict(os.environ, GQ_LIB=lib))
    a = {(r[0], r[1], r[2]): r for r in json.load(open("gpurun_out/sd_old.json"))}
    b = {(r[0], r[1], r[2]): r for r in json.load(open("gpurun_out/sd_new.json"))}
    only_a, only_b = sorted(set(a) - set(b)), sorted(set(b) - set(a))
    print("old %d new %d only_old %d only_new %d" % (len(a), len(b), len(only_a), len(only_b)))
    for k in only_a:
        print("old only", a[k])
    for k in only_b:
        print("new only", b[k])
    # the oracle at each differing locus (window of 1 locus, reads overlapping it)
    from guacamole_amd import synthetic
    from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
    from oracle import oracle as O
    L = int(os.environ.get("SD_LENGTH", CHR20))
    seed = synthetic.SEED + 3
    tg = synthetic.generate(L, 60.0, seed=seed, somatic_rate=2e-4, tumor=True, read_seed=11)
    ng = synthetic.generate(L, 30.0, seed=seed, somatic_rate=2e-4, tumor=False, read_seed=12)
    for k in only_a + only_b:
        pos = k[0]
        rt, rn = tg.to_read_set(tg.window(pos, pos + 1)), ng.to_read_set(ng.window(pos, pos + 1))
        ls = LociSet.parse("%s:%d-%d" % (rt.contig_names[0], pos, pos + 1)).result(rt.contig_lengths_map)
        want = O.somatic_standard(rt, rn, flatten_partitions(partition_loci_uniformly(1, ls), rt.contig_index()))
        print("oracle at", pos, [(r["ref"], r["alt"], r["log_odds"], r["gq"], r["flags"]) for r in want])


if __name__ == "__main__":
    main()
