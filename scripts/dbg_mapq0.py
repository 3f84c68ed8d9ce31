import sys, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
from guacamole_amd.synthetic import generate
from oracle import oracle as O
L = 200_000
tg = generate(L, 60.0, seed=20261015 + 3, somatic_rate=2e-4, tumor=True, read_seed=41)
ng = generate(L, 30.0, seed=20261015 + 3, somatic_rate=2e-4, tumor=False, read_seed=42)
t, n = tg.to_read_set(), ng.to_read_set()
for locus in (11878,):
    m = (t.start <= locus) & (t.end > locus)
    idx = np.nonzero(m)[0]
    print("tumor depth", len(idx), "mapq", sorted(t.mapq[idx].tolist()))
    bases = [chr(t.seq[t.seq_off[i] + (locus - t.start[i])]) for i in idx]
    print("bases", "".join(bases))
    loci = (np.array([0], np.int32), np.array([locus], np.int64), np.array([locus + 1], np.int64), np.array([0], np.int64))
    print(O.somatic_standard(t, n, loci, min_mapq=0, apply_filters=0))
