"""Helper for tests/test_gpu_variants.py (run as a script on the GPU box): one process's somatic
and germline records over a synthetic 60x / 30x pair, printed as one JSON line.  The kernel
variants the library picks from the environment once per process (GQ_CALL_SPLIT, GQ_CALL_WPE,
GQ_FILL_U) are compared across processes by the test."""
import hashlib
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from guacamole_amd import native, synthetic  # noqa: E402


def digest(obj) -> str:
    def norm(x):
        if isinstance(x, float) and math.isnan(x):
            return "nan"
        if isinstance(x, float):
            return x.hex()
        if isinstance(x, (list, tuple)):
            return [norm(y) for y in x]
        if isinstance(x, dict):
            return {k: norm(v) for k, v in sorted(x.items())}
        return x
    return hashlib.sha256(json.dumps(norm(obj), sort_keys=True).encode()).hexdigest()


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000
    seed = synthetic.SEED + 3
    tg = synthetic.generate(L, 60.0, seed=seed, somatic_rate=2e-3, tumor=True, read_seed=11)
    ng = synthetic.generate(L, 30.0, seed=seed, somatic_rate=2e-3, tumor=False, read_seed=12)
    ctx = native.Context(0)
    t = ctx.upload(tg.arrays)
    n = ctx.upload(ng.arrays)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([L - 1], np.int64), np.array([0], np.int64))
    som = ctx.somatic_standard(t, n, loci).rows
    germ = ctx.germline_threshold(t, loci, 8, False, False).tuples(["20"])
    print(json.dumps({"somatic": len(som), "somatic_digest": digest(som), "germline": len(germ),
                      "germline_digest": digest([list(map(str, r)) for r in germ])}))


if __name__ == "__main__":
    main()
